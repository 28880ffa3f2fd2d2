#!/usr/bin/env python3
"""Which path tkv_wal_verify takes on a 1 GiB WAL of small records, and how long each part takes."""
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
last = np.zeros(4, np.uint64)


def run(tag, fn):
    for r in range(3):
        t0 = time.perf_counter()
        res = fn()
        dt = time.perf_counter() - t0
        lib.tkv_debug_wal_last(last.ctypes.data)
        print(f"{tag}: {res} {dt * 1e3:.1f} ms  passes={last[0]} host_walk={last[1]} copied={last[2]} pieces={last[3]}",
              flush=True)


run("host pageable", lambda: tk.wal.verify(w))
d = torch.from_numpy(w).cuda()
run("device", lambda: tk.wal.verify_device(d))
t0 = time.perf_counter()
d2 = torch.from_numpy(w).cuda()
torch.cuda.synchronize()
print(f"plain torch H2D of the image: {(time.perf_counter() - t0) * 1e3:.1f} ms")

# the formats bench's 430 MB image (Zipf values up to 16 KB), device-resident, for the kernel profile
rng = np.random.default_rng(1)
n_rec = 400_000
klen = rng.integers(8, 64, n_rec).astype(np.uint32)
vlen = np.minimum(rng.zipf(1.6, n_rec) * 64, 16_000).astype(np.uint32)
size = 26 + klen + vlen
offs = np.concatenate([[0], np.cumsum(size[:-1], dtype=np.uint64)]).astype(np.uint64)
total = int(size.sum())
wal = rng.integers(0, 256, total, dtype=np.uint8)
for col, vals in ((0, size - 8), (18, klen), (22, vlen)):
    for b in range(4):
        wal[offs.astype(np.int64) + col + b] = ((vals >> (8 * b)) & 0xFF).astype(np.uint8)
for col in (8, 17):
    wal[offs.astype(np.int64) + col] = 0
s32 = size.astype(np.uint32)
tk.check(lib.tkv_wal_stamp(ctypes.c_void_p(wal.ctypes.data), ctypes.c_void_p(offs.ctypes.data),
                           ctypes.c_void_p(s32.ctypes.data), n_rec))
dz = torch.from_numpy(wal).cuda()
run("zipf device", lambda: tk.wal.verify_device(dz))
run("zipf host pageable", lambda: tk.wal.verify(wal))
