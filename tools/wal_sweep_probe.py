#!/usr/bin/env python3
"""Probe (not product code): the device WAL verify on the 1 GiB image of small records and the 430 MB
Zipf image (tools/ab_wal.py's images), timed per call, for rocprofv3 kernel traces of its kernels.

    python tools/wal_sweep_probe.py [lib.so] [--reps 10] [--image small|zipf|both|adv|advgiant]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from ab_wal import image  # noqa: E402

VP, U64 = ctypes.c_void_p, ctypes.c_uint64


def adversarial(rng, target=1 << 30, giant=0.0):
    """Zipf values (|v| = min(48 zipf(1.6), 16000)), every value a run of well-formed 40-byte records
    (tests/test_gpu_wal_device.py::test_values_made_of_records at 1 GiB): every chunk and search start
    inside a value lands on a fake chain. giant: the share of values given 1-4 MiB (also runs of fake
    records), so that most chunk boundaries fall inside a giant record."""
    n = int(target / 300)
    klen = rng.integers(0, 40, n).astype(np.uint32)
    vlen = np.minimum(rng.zipf(1.6, n) * 48, 16000).astype(np.uint32)
    if giant:
        g = rng.random(n) < giant
        vlen[g] = rng.integers(1 << 20, 4 << 20, int(g.sum())).astype(np.uint32)
    size = 26 + klen.astype(np.uint64) + vlen
    n = int(np.searchsorted(np.cumsum(size), target))
    klen, vlen, size = klen[:n], vlen[:n], size[:n]
    w, offs, sz = image(n, klen, vlen, rng)
    fake = np.zeros(40, np.uint8)
    fake[0:4] = np.frombuffer((32).to_bytes(4, "little"), np.uint8)
    fake[18:22] = np.frombuffer((6).to_bytes(4, "little"), np.uint8)
    fake[22:26] = np.frombuffer((8).to_bytes(4, "little"), np.uint8)
    v0 = (offs + 26 + klen).astype(np.int64)
    ln = (vlen // 40 * 40).astype(np.int64)
    for a in range(0, n, 200_000):
        b = min(n, a + 200_000)
        L = ln[a:b]
        tot = int(L.sum())
        if not tot:
            continue
        start = np.repeat(v0[a:b], L)
        r = np.arange(tot, dtype=np.int64) - np.repeat(np.cumsum(L) - L, L)
        w[start + r] = fake[r % 40]
    return w, offs, sz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=os.path.join(ROOT, "tinykvpp_amd", "libtkv_crc32.so"))
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--image", default="both")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    lib = ctypes.CDLL(os.path.abspath(args.lib))
    lib.tkv_wal_verify_device.argtypes = [VP, U64, ctypes.POINTER(U64), ctypes.POINTER(U64), VP]
    lib.tkv_wal_stamp.argtypes = [VP, VP, VP, U64]
    lib.tkv_debug_wal_last.argtypes = [VP]
    assert lib.tkv_set_device(0) == 0
    rng = np.random.default_rng(1)
    imgs = []
    if args.image in ("small", "both"):
        n = 18_199_191
        imgs.append(("small records 1 GiB", image(n, rng.integers(4, 24, n).astype(np.uint32),
                                                  rng.integers(0, 40, n).astype(np.uint32), rng)))
    if args.image == "adv":
        imgs.append(("values made of records 1 GiB", adversarial(rng)))
    if args.image == "advgiant":
        imgs.append(("values made of records, 0.1 % of 1-4 MiB, 1 GiB", adversarial(rng, giant=0.001)))
    if args.image in ("zipf", "both"):
        n2 = 400_000
        imgs.append(("zipf 430 MB", image(n2, rng.integers(8, 64, n2).astype(np.uint32),
                                          np.minimum(rng.zipf(1.6, n2) * 64, 16_000).astype(np.uint32), rng)))
    st = VP(torch.cuda.current_stream().cuda_stream)
    for name, (w, offs, sz) in imgs:
        assert lib.tkv_wal_stamp(VP(w.ctypes.data), VP(offs.ctypes.data), VP(sz.ctypes.data), offs.size) == 0
        d = torch.from_numpy(w).cuda()
        torch.cuda.synchronize()
        stamps = hasattr(lib, "tkv_debug_wal_stamps")
        sv = np.zeros(8, np.uint64)
        if hasattr(lib, "tkv_debug_wal_rounds"):
            lib.tkv_debug_wal_rounds.restype = ctypes.c_size_t
            lib.tkv_debug_wal_rounds.argtypes = [VP, ctypes.c_size_t]
            rw = np.zeros(6 * 256, np.uint64)
            k = lib.tkv_debug_wal_rounds(VP(rw.ctypes.data), rw.size)
            rounds = [dict(zip(("failing", "tasks", "longest", "regions", "walk_max", "walked"), map(int, rw[i:i + 6])))
                      for i in range(0, min(k, rw.size), 6)]
            if rounds:
                print(json.dumps({"image": name, "fixup_rounds": rounds}), flush=True)
        if stamps:
            lib.tkv_debug_wal_stamps(VP(sv.ctypes.data))
        ts = []
        for r in range(args.reps + 1):
            good, stop = U64(0), U64(0)
            t0 = time.perf_counter()
            rc = lib.tkv_wal_verify_device(VP(d.data_ptr()), w.size, ctypes.byref(good), ctypes.byref(stop), st)
            dt = time.perf_counter() - t0
            print(json.dumps({"image": name, "rep": r, "ms": round(dt * 1e3, 3)}), flush=True)
            assert rc == 0 and good.value == offs.size and stop.value == w.size, (rc, good.value, stop.value)
            if r:
                ts.append(dt)
        last = np.zeros(4, np.uint64)
        lib.tkv_debug_wal_last(VP(last.ctypes.data))
        med = float(np.median(ts))
        print(json.dumps({"image": name, "bytes": int(w.size), "records": int(offs.size), "median_ms": round(med * 1e3, 3),
                          "min_ms": round(min(ts) * 1e3, 3), "GB_per_s": round(w.size / med / 1e9, 1), "rounds": int(last[0]),
                          "host_walk": int(last[1]), "fixup_free": int(last[3])}),
              flush=True)
        if hasattr(lib, "tkv_debug_wal_rounds"):
            lib.tkv_debug_wal_rounds.restype = ctypes.c_size_t
            lib.tkv_debug_wal_rounds.argtypes = [VP, ctypes.c_size_t]
            rw = np.zeros(6 * 256, np.uint64)
            k = lib.tkv_debug_wal_rounds(VP(rw.ctypes.data), rw.size)
            rounds = [dict(zip(("failing", "tasks", "longest", "regions", "walk_max", "walked"), map(int, rw[i:i + 6])))
                      for i in range(0, min(k, rw.size), 6)]
            if rounds:
                print(json.dumps({"image": name, "fixup_rounds": rounds}), flush=True)
        if stamps:
            lib.tkv_debug_wal_stamps(VP(sv.ctypes.data))
            names = ["put", "search", "walk", "link", "list", "fold", "record"]
            tot = float(sv[:7].sum())
            print(json.dumps({"image": name, "regions": int(sv[7]), "cycles_per_region": round(tot / max(int(sv[7]), 1), 1),
                              "share": {n: round(float(sv[i]) / tot, 3) for i, n in enumerate(names)}}), flush=True)


if __name__ == "__main__":
    main()
