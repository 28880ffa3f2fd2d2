#!/usr/bin/env python3
"""In-process comparison of builds of libtkv_crc32.so on the device WAL verify (not product code):
the 1 GiB image of small records (tools/wal_dev_probe.py) and the formats bench's 430 MB Zipf image,
resident in HBM; every library verifies each image in rotation, results must agree.

    python tools/ab_wal.py lib1.so lib2.so ... [--rounds 6]
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
VP, U64 = ctypes.c_void_p, ctypes.c_uint64


def image(n_rec, klen, vlen, rng):
    size = 26 + klen + vlen
    offs = np.concatenate([[0], np.cumsum(size[:-1], dtype=np.uint64)]).astype(np.uint64)
    w = rng.integers(0, 256, int(size.sum()), dtype=np.uint8)
    for col, vals in ((0, size - 8), (18, klen), (22, vlen)):
        for b in range(4):
            w[offs.astype(np.int64) + col + b] = ((vals >> (8 * b)) & 0xFF).astype(np.uint8)
    for col in (8, 17):
        w[offs.astype(np.int64) + col] = 0
    return w, offs, size.astype(np.uint32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=6)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    libs = []
    for p in args.libs:
        lib = ctypes.CDLL(os.path.abspath(p))
        lib.tkv_wal_verify_device.argtypes = [VP, U64, ctypes.POINTER(U64), ctypes.POINTER(U64), VP]
        lib.tkv_wal_stamp.argtypes = [VP, VP, VP, U64]
        assert lib.tkv_set_device(0) == 0
        libs.append(lib)
    rng = np.random.default_rng(1)
    n = 18_199_191
    small = image(n, rng.integers(4, 24, n).astype(np.uint32), rng.integers(0, 40, n).astype(np.uint32), rng)
    n2 = 400_000
    zipf = image(n2, rng.integers(8, 64, n2).astype(np.uint32),
                 np.minimum(rng.zipf(1.6, n2) * 64, 16_000).astype(np.uint32), rng)
    st = VP(torch.cuda.current_stream().cuda_stream)
    for name, (w, offs, sz) in (("small records 1 GiB", small), ("zipf 430 MB", zipf)):
        assert libs[0].tkv_wal_stamp(VP(w.ctypes.data), VP(offs.ctypes.data), VP(sz.ctypes.data), offs.size) == 0
        d = torch.from_numpy(w).cuda()
        torch.cuda.synchronize()
        times = [[] for _ in libs]
        res = [None] * len(libs)
        for r in range(args.rounds):
            for k in (list(range(len(libs)))[r % len(libs):] + list(range(len(libs)))[:r % len(libs)]):
                good, stop = U64(0), U64(0)
                t0 = time.perf_counter()
                rc = libs[k].tkv_wal_verify_device(VP(d.data_ptr()), w.size, ctypes.byref(good), ctypes.byref(stop), st)
                dt = time.perf_counter() - t0
                res[k] = (rc, good.value, stop.value)
                if r:
                    times[k].append(dt)
        for k, p in enumerate(args.libs):
            med = float(np.median(times[k]))
            print(json.dumps({"image": name, "lib": os.path.basename(p), "median_ms": round(med * 1e3, 3),
                              "GB_per_s": round(w.size / med / 1e9, 1), "result": res[k],
                              "same_as_first": res[k] == res[0]}), flush=True)


if __name__ == "__main__":
    main()
