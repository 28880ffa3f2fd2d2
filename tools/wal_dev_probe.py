#!/usr/bin/env python3
"""Device WAL verify alone (tkv_wal_verify_device) on the 1 GiB image of small records that
tools/wal_probe.py builds, three times: a short program for kernel traces and PMC passes."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tinykvpp_amd as tk  # noqa: E402

torch.cuda.set_device(0)
tk.set_device(0)
lib = tk.load_library()
rng = np.random.default_rng(1)
sk = rng.integers(4, 24, 20_000_000).astype(np.uint32)
sv = rng.integers(0, 40, 20_000_000).astype(np.uint32)
ssz = 26 + sk + sv
n = int(np.searchsorted(np.cumsum(ssz, dtype=np.uint64), np.uint64(1 << 30)))
sk, sv, ssz = sk[:n], sv[:n], ssz[:n]
offs = np.concatenate([[0], np.cumsum(ssz[:-1], dtype=np.uint64)]).astype(np.uint64)
total = int(ssz.sum())
w = rng.integers(0, 256, total, dtype=np.uint8)
for col, vals in ((0, ssz - 8), (18, sk), (22, sv)):
    for b in range(4):
        w[offs.astype(np.int64) + col + b] = ((vals >> (8 * b)) & 0xFF).astype(np.uint8)
for col in (8, 17):
    w[offs.astype(np.int64) + col] = 0
s32 = ssz.astype(np.uint32)
tk.check(lib.tkv_wal_stamp(ctypes.c_void_p(w.ctypes.data), ctypes.c_void_p(offs.ctypes.data),
                           ctypes.c_void_p(s32.ctypes.data), n))
d = torch.from_numpy(w).cuda()
for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    t0 = time.perf_counter()
    res = tk.wal.verify_device(d)
    print(f"device: {res} {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
