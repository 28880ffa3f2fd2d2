#!/usr/bin/env python3
"""Probe (not product code): the device WAL verify on the 1 GiB image of small records and the 430 MB
Zipf image (tools/ab_wal.py's images), timed per call, for rocprofv3 kernel traces of its kernels.

    python tools/wal_sweep_probe.py [lib.so] [--reps 10] [--image small|zipf|both]
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
        if stamps:
            lib.tkv_debug_wal_stamps(VP(sv.ctypes.data))
        ts = []
        for r in range(args.reps + 1):
            good, stop = U64(0), U64(0)
            t0 = time.perf_counter()
            rc = lib.tkv_wal_verify_device(VP(d.data_ptr()), w.size, ctypes.byref(good), ctypes.byref(stop), st)
            dt = time.perf_counter() - t0
            assert rc == 0 and good.value == offs.size and stop.value == w.size, (rc, good.value, stop.value)
            if r:
                ts.append(dt)
        last = np.zeros(4, np.uint64)
        lib.tkv_debug_wal_last(VP(last.ctypes.data))
        med = float(np.median(ts))
        print(json.dumps({"image": name, "median_ms": round(med * 1e3, 3), "min_ms": round(min(ts) * 1e3, 3),
                          "GB_per_s": round(w.size / med / 1e9, 1), "rounds": int(last[0]), "fixup_free": int(last[3])}),
              flush=True)
        if stamps:
            lib.tkv_debug_wal_stamps(VP(sv.ctypes.data))
            names = ["put", "search", "walk", "link", "list", "fold", "record"]
            tot = float(sv[:7].sum())
            print(json.dumps({"image": name, "regions": int(sv[7]), "cycles_per_region": round(tot / max(int(sv[7]), 1), 1),
                              "share": {n: round(float(sv[i]) / tot, 3) for i, n in enumerate(names)}}), flush=True)


if __name__ == "__main__":
    main()
