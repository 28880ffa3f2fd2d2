#!/usr/bin/env python3
"""WAL-record-sized blocks (not product code): several builds of libtkv_crc32.so in one process,
rotated round by round on one stream and the same device buffers. GB/s of payload from HIP events
around K launches (median over rounds); every library's results are checked against the first's.

    python tools/lane_probe.py lib1.so [lib2.so ...] [--rounds 5] [--reps 5] [--gib 1] [--only 36]

Workloads: uniform batches of 26-64 B blocks and of 65 B - 2 KiB blocks (the reference's records are
26 + |k| + |v| bytes, wal.cpp:25), the same at the WAL payload pitch (8-byte header between payloads)
and at an odd base, and irregular batches of WAL payloads (8-byte gaps), back-to-back small blocks
and a mixed 0-4 KiB batch.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

VP = ctypes.c_void_p
U64 = ctypes.c_uint64


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    lib.tkv_crc32_batch_uniform_device.argtypes = [VP, U64, U64, VP, VP, U64, VP]
    lib.tkv_crc32_batch_device.argtypes = [VP, VP, VP, VP, VP, U64, VP]
    lib.tkv_last_error.restype = ctypes.c_char_p
    assert lib.tkv_set_device(0) == 0
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--gib", type=float, default=1.0)
    ap.add_argument("--only", default=None)
    ap.add_argument("--lens", default=None, help="comma-separated uniform lengths instead of the default list")
    ap.add_argument("--init", action="store_true", help="uniform batches with per-block initial registers")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    libs = [load(p) for p in args.libs]
    st = torch.cuda.current_stream()
    sp = VP(st.cuda_stream)
    total = int(args.gib * (1 << 30))
    data = torch.randint(0, 256, (total + (total // 4) + 8192,), dtype=torch.uint8, device="cuda")
    D = data.data_ptr()
    rng = np.random.default_rng(0)

    def uniform(L, stride=None, off=0):
        stride = stride or L
        n = total // stride
        ini = torch.randint(0, 2**31 - 1, (n,), dtype=torch.int32, device="cuda") if args.init else None
        iv = VP(ini.data_ptr()) if args.init else None
        return (f"uniform {L} B stride {stride} base+{off}" + (" per-block init" if args.init else ""), n * L, n,
                lambda lib, o: lib.tkv_crc32_batch_uniform_device(VP(D + off), stride, L, iv, o, n, sp))

    def irregular(name, lens, gaps, off=0):
        lens = np.asarray(lens, np.int64)
        offs = off + np.concatenate([[0], np.cumsum(lens[:-1] + gaps[:-1])])
        d_o = torch.from_numpy(offs.astype(np.int64)).cuda()
        d_l = torch.from_numpy(lens.astype(np.int32)).cuda()
        n = lens.size
        return (name, int(lens.sum()), n,
                lambda lib, o: lib.tkv_crc32_batch_device(VP(D), VP(d_o.data_ptr()), VP(d_l.data_ptr()), None, o, n, sp),
                (d_o, d_l))

    def count(L, pitch):
        return total // pitch

    work = []
    for L in ([int(x) for x in args.lens.split(",")] if args.lens else (16, 26, 28, 32, 33, 36, 48, 59, 64)):
        work.append(uniform(L))
    for L in (100, 200, 300, 500, 1000, 1500, 2000):  # 65 B - 2 KiB, not multiples of 16 (crc_packed_small_gen)
        work.append(uniform(L))
    work.append(uniform(512, 512, 3))  # a multiple of 16 at an odd base
    work.append(uniform(256, 264, 8))  # WAL payload pitch
    work.append(uniform(36, 44, 8))   # WAL payload pitch: 8-byte header in front of every 36-byte payload
    work.append(uniform(36, 36, 3))   # odd base
    work.append(uniform(59, 67, 8))
    n36 = count(36, 44)
    work.append(irregular("irregular WAL payloads 36 B, 8 B gaps", np.full(n36, 36), np.full(n36, 8), 8))
    nm = count(42, 50)
    lm = rng.choice([26, 28, 33, 36, 59], nm)
    work.append(irregular("irregular WAL payloads 26-59 B, 8 B gaps", lm, np.full(nm, 8), 8))
    nm = count(45, 53)  # mostly lane blocks, 2 % longer values (one-pass packed kernel)
    lm = np.where(rng.random(nm) < 0.02, rng.integers(65, 401, nm), rng.choice([26, 28, 33, 36, 59], nm))
    work.append(irregular("irregular WAL payloads 26-59 B + 2 % 65-400 B, 8 B gaps", lm, np.full(nm, 8), 8))
    ng = count(150, 158)
    work.append(irregular("irregular WAL payloads 100-200 B, 8 B gaps", rng.integers(100, 201, ng), np.full(ng, 8), 8))
    ng = count(160, 168)
    work.append(irregular("irregular WAL payloads 65-256 B, 8 B gaps", rng.integers(65, 257, ng), np.full(ng, 8), 8))
    ng = count(128, 136)
    work.append(irregular("irregular 128 B, 8 B gaps", np.full(ng, 128), np.full(ng, 8), 8))
    n = count(36, 36)
    work.append(irregular("irregular back to back 36 B", np.full(n, 36), np.zeros(n, np.int64), 0))
    n = count(64, 64)
    work.append(irregular("irregular back to back 64 B", np.full(n, 64), np.zeros(n, np.int64), 0))
    n = count(128, 128)
    work.append(irregular("irregular back to back 128 B", np.full(n, 128), np.zeros(n, np.int64), 0))
    n = count(150, 150)
    work.append(irregular("irregular back to back 100-200 B", rng.integers(100, 201, n), np.zeros(n, np.int64), 0))
    # 257 B - 1 KiB: WAL payloads with mid-size values, gapped and back to back
    for lo, hi in ((257, 512), (513, 1024), (300, 1000), (257, 1024)):
        ng = count((lo + hi) // 2, (lo + hi) // 2 + 8)
        work.append(irregular(f"irregular {lo}-{hi} B, 8 B gaps", rng.integers(lo, hi + 1, ng), np.full(ng, 8), 8))
    ng = count(650, 650)
    work.append(irregular("irregular back to back 300-1000 B", rng.integers(300, 1001, ng), np.zeros(ng, np.int64), 0))
    ng = count(512, 520)
    work.append(irregular("irregular 0-1024 B, 8 B gaps", rng.integers(0, 1025, ng), np.full(ng, 8), 8))
    ng = count(450, 458)
    work.append(irregular("irregular 200-700 B, 8 B gaps", rng.integers(200, 701, ng), np.full(ng, 8), 8))
    ng = count(400, 408)  # group-pass densities between the thresholds: 65-256 B ~26 %, 257-512 B ~43 %
    work.append(irregular("irregular 100-700 B, 8 B gaps", rng.integers(100, 701, ng), np.full(ng, 8), 8))
    ng = count(290, 298)  # 65-256 B ~40 %, 257-512 B ~60 %
    work.append(irregular("irregular 180-400 B, 8 B gaps", rng.integers(180, 401, ng), np.full(ng, 8), 8))
    ng = count(300, 308)  # listed 257-384 B (the 8-lane pass needs 3968 of 4096 per tile)
    lm = np.where(rng.random(ng) < 0.1, rng.integers(100, 201, ng), rng.integers(257, 385, ng))
    work.append(irregular("irregular 257-384 B + 10 % 100-200 B, 8 B gaps", lm, np.full(ng, 8), 8))
    ng = count(545, 553)
    work.append(irregular("irregular 65-1024 B, 8 B gaps", rng.integers(65, 1025, ng), np.full(ng, 8), 8))
    n = count(2048, 2056)
    lr = rng.integers(0, 4097, n)
    work.append(irregular("irregular 0-4 KiB, 8 B gaps", lr, np.full(n, 8), 8))

    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for w in work:
        name, nbytes, n, call = w[0], w[1], w[2], w[3]
        if args.only and args.only not in name:
            continue
        outs = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in libs]
        times = [[] for _ in libs]
        for r in range(args.rounds):
            for k in range(len(libs)):
                i = (k + r) % len(libs)
                call(libs[i], VP(outs[i].data_ptr()))
                torch.cuda.synchronize()
                e0.record(st)
                for _ in range(args.reps):
                    rc = call(libs[i], VP(outs[i].data_ptr()))
                e1.record(st)
                torch.cuda.synchronize()
                if rc != 0:
                    raise SystemExit(f"{args.libs[i]}: {name}: rc {rc}: {libs[i].tkv_last_error()}")
                times[i].append(e0.elapsed_time(e1) / args.reps)
        for i, p in enumerate(args.libs):
            ms = float(np.median(times[i]))
            same = bool(torch.equal(outs[i], outs[0]))
            print(json.dumps({"work": name, "lib": os.path.basename(p), "blocks": n, "payload_bytes": nbytes,
                              "ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1), "same_as_first": same}),
                  flush=True)
        del outs


if __name__ == "__main__":
    main()
