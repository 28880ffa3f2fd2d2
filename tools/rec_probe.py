#!/usr/bin/env python3
"""WAL record-list check against the generic irregular batch on the same records (not product code).

Images of ~1 GiB in HBM laid out as wal.cpp:19-61 (stamped by tkv_wal_stamp):
  * "36 B payloads": uniform 44-byte records (payload 36 B, the verdict's gapped WAL payloads);
  * "28 B payloads": uniform 36-byte records (the shape round 4's first probes ran under the 36 B label);
  * "small records": 26 + |k| + |v| bytes, |k| 4-23, |v| 0-39 (tools/ab_wal.py's image, payloads 22-80 B).
For each: tkv_wal_check_records_device over the record offsets (u32) and tkv_crc32_batch_device over
(payload offsets u64, lengths u32), HIP events around K calls, several libraries rotated in one
process. GB/s are payload bytes; results are checked against the first library and the stored CRCs.

    python tools/rec_probe.py lib1.so [lib2.so ...] [--rounds 5] [--reps 5] [--only 36]
"""
import argparse
import ctypes
import json
import os

import numpy as np
import torch

VP, U64, U32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    lib.tkv_crc32_batch_device.argtypes = [VP, VP, VP, VP, VP, U64, VP]
    lib.tkv_wal_stamp.argtypes = [VP, VP, VP, U64]
    lib.tkv_last_error.restype = ctypes.c_char_p
    if hasattr(lib, "tkv_wal_check_records_device"):
        lib.tkv_wal_check_records_device.argtypes = [VP, U64, VP, U64, U32, VP, VP, VP]
    assert lib.tkv_set_device(0) == 0
    return lib


def image(lib, klen, vlen, rng):
    size = 26 + klen + vlen
    offs = np.concatenate([[0], np.cumsum(size[:-1], dtype=np.uint64)]).astype(np.uint64)
    w = rng.integers(0, 256, int(size.sum()), dtype=np.uint8)
    for col, vals in ((0, size - 8), (18, klen), (22, vlen)):
        for b in range(4):
            w[offs.astype(np.int64) + col + b] = ((vals >> (8 * b)) & 0xFF).astype(np.uint8)
    s32 = size.astype(np.uint32)
    assert lib.tkv_wal_stamp(VP(w.ctypes.data), VP(offs.ctypes.data), VP(s32.ctypes.data), offs.size) == 0
    return w, offs, size


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--gib", type=float, default=1.0)
    ap.add_argument("--only", default=None)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    libs = [load(p) for p in args.libs]
    st = torch.cuda.current_stream()
    sp = VP(st.cuda_stream)
    rng = np.random.default_rng(1)
    total = int(args.gib * (1 << 30))
    n36 = total // 44
    n_small = total // 59
    # (round 4's first probes used klen 4 / vlen 6, i.e. 36-byte records with 28-byte payloads, under
    # the 36 B label; both shapes are measured now)
    n28 = total // 36
    imgs = [("36 B payloads (44-byte records)", np.full(n36, 8, np.uint64), np.full(n36, 10, np.uint64), 36),
            ("28 B payloads (36-byte records)", np.full(n28, 4, np.uint64), np.full(n28, 6, np.uint64), 28),
            ("small records (payloads 22-80 B)", rng.integers(4, 24, n_small).astype(np.uint64),
             rng.integers(0, 40, n_small).astype(np.uint64), 80)]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, klen, vlen, maxp in imgs:
        if args.only and args.only not in name:
            continue
        w, offs, size = image(libs[0], klen, vlen, rng)
        n = offs.size
        d = torch.from_numpy(w).cuda()
        d_roff = torch.from_numpy(offs.astype(np.uint32).view(np.int32)).cuda()
        d_poff = torch.from_numpy((offs + 8).astype(np.int64)).cuda()
        d_plen = torch.from_numpy((size - 8).astype(np.int32)).cuda()
        stored = w[(offs[:, None].astype(np.int64) + np.arange(4, 8))].copy().view("<u4").reshape(-1)
        payload = int((size - 8).sum())
        del w
        fb = torch.empty(1, dtype=torch.int64, device="cuda")
        calls = [("check_records", lambda lib, o: lib.tkv_wal_check_records_device(
                     VP(d.data_ptr()), d.numel(), VP(d_roff.data_ptr()), n, maxp, o, VP(fb.data_ptr()), sp)),
                 ("batch_device", lambda lib, o: lib.tkv_crc32_batch_device(
                     VP(d.data_ptr()), VP(d_poff.data_ptr()), VP(d_plen.data_ptr()), None, o, n, sp))]
        for cname, call in calls:
            outs = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in libs]
            times = [[] for _ in libs]
            usable = [cname != "check_records" or hasattr(lib, "tkv_wal_check_records_device") for lib in libs]
            for r in range(args.rounds):
                for k in range(len(libs)):
                    i = (k + r) % len(libs)
                    if not usable[i]:
                        continue
                    call(libs[i], VP(outs[i].data_ptr()))
                    torch.cuda.synchronize()
                    e0.record(st)
                    for _ in range(args.reps):
                        rc = call(libs[i], VP(outs[i].data_ptr()))
                    e1.record(st)
                    torch.cuda.synchronize()
                    if rc != 0:
                        raise SystemExit(f"{args.libs[i]}: {name} {cname}: rc {rc}: {libs[i].tkv_last_error()}")
                    times[i].append(e0.elapsed_time(e1) / args.reps)
            for i, p in enumerate(args.libs):
                if not usable[i]:
                    continue
                ms = float(np.median(times[i]))
                got = outs[i].cpu().numpy().view(np.uint32)
                rec = {"image": name, "call": cname, "lib": os.path.basename(p), "records": n,
                       "payload_bytes": payload, "image_bytes": d.numel(), "ms": round(ms, 4),
                       "payload_GBps": round(payload / ms / 1e6, 1), "image_GBps": round(d.numel() / ms / 1e6, 1),
                       "crc_equal_stored": bool(np.array_equal(got, stored))}
                if cname == "check_records":
                    rec["first_bad"] = int(fb.item())
                print(json.dumps(rec), flush=True)
            del outs
        del d, d_roff, d_poff, d_plen
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
