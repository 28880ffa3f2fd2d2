#!/usr/bin/env python3
"""Reproduce one test_wal_verify_random case (not product code): rebuild the image of a seed and run
the host-image path and the device-image path at every base shift 0..15, against the sequential
decode."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import tinykvpp_amd as tk  # noqa: E402
from conftest import Oracle  # noqa: E402
from test_gpu_wal_device import both, make_wal, sequential_decode  # noqa: E402

seed = int(sys.argv[1])
if len(sys.argv) > 2:
    tk.load_library(os.path.abspath(sys.argv[2]))  # a probe build instead of the product library
torch.cuda.set_device(0)
tk.set_device(0)
oracle = Oracle(os.path.join(ROOT, "oracle", "liboracle.so"))
rng = np.random.default_rng(4000 + seed)
n_rec = int(rng.choice([1, 2, 7, 300, 5000, 20000, 120000]))
vmax = int(rng.choice([64, 600, 5000, 16000])) if n_rec < 100000 else 600
img, offs, size = make_wal(rng, n_rec, vmax=vmax, fake_headers=float(rng.choice([0.0, 0.0, 0.3])))
kind = ("none", "payload", "crc", "record_len", "kv_overflow", "any")[seed % 6]
r = int(rng.integers(0, n_rec))
o = int(offs[r])
print("n_rec", n_rec, "sizes", size[:8], "offs", offs[:8], "kind", kind, "record", r, flush=True)
if kind == "kv_overflow":
    img[o + 22:o + 26] = np.frombuffer((int(size[r])).to_bytes(4, "little"), np.uint8)
    lib = tk.load_library()
    one_off = np.array([o], np.uint64)
    one_len = np.array([int(size[r])], np.uint32)
    tk.check(lib.tkv_wal_stamp(ctypes.c_void_p(img.ctypes.data), ctypes.c_void_p(one_off.ctypes.data),
                               ctypes.c_void_p(one_len.ctypes.data), 1))
n = img.size if rng.random() < 0.6 else int(rng.integers(0, img.size + 1))
shift0 = int(rng.integers(0, 16))
want = sequential_decode(oracle, img, n)
print("n", n, "want", want, "test shift", shift0, flush=True)
for shift in range(16):
    got = both(img, n, shift=shift)
    print(shift, got, "OK" if got == (want, want) else "MISMATCH", flush=True)

# the engine alone: one block [8, 8 + L) of a base shifted by 0..15 bytes
for L in (5031, 94, 1025, 4096, 4097, 8000):
    bad = []
    for shift in range(16):
        host = np.random.default_rng(L + shift).integers(0, 256, 8 + L + 64, dtype=np.uint8)
        d = torch.zeros(host.size + shift, dtype=torch.uint8, device="cuda")
        d[shift:] = torch.from_numpy(host).cuda()
        got = tk.crc32_batch(d[shift:], torch.tensor([8], dtype=torch.int64, device="cuda"),
                             torch.tensor([L], dtype=torch.int32, device="cuda"))
        want = oracle.batch(host, np.array([8], np.uint64), np.array([L], np.uint32))
        if int(got.cpu().numpy().view(np.uint32)[0]) != int(want[0]):
            bad.append(shift)
    print("engine one block L", L, "bad shifts", bad, flush=True)
