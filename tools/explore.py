#!/usr/bin/env python3
"""A/B the row-kernel variants of tools/libexplore.so in one process (interleaved rounds) on the
cfg2 (1 M x 4 KiB) or cfg3 (256 K x 64 KiB) buffer; prints median/min GB/s per variant and checks the
CRC variants against the product library's output."""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tinykvpp_amd as tk  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--len", type=int, default=4096)
ap.add_argument("--gib", type=float, default=4.0)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--only", default="")
ap.add_argument("--zero", action="store_true", help="zero-filled buffer (data-dependent power / clock probe)")
ap.add_argument("--irregular", action="store_true", help="cfg4 Zipf batch through the irregular-kernel variants")
a = ap.parse_args()

lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libexplore.so"))
lib.explore_name.restype = ctypes.c_char_p
lib.explore_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p,
                            ctypes.c_void_p]
nv = lib.explore_count()
names = [lib.explore_name(i).decode() for i in range(nv)]
sel = [i for i in range(nv) if not a.only or any(s in names[i] for s in a.only.split(","))]

torch.cuda.set_device(0)
tk.set_device(0)
if a.irregular:
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from conftest import Oracle
    ora = Oracle(os.path.join(ROOT, "oracle", "liboracle.so"))
    lens = ora.zipf_lengths(1, 0, 1 << 17)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
    total = int(lens.sum())
    data = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    d_off = torch.from_numpy(offs).to("cuda")
    d_len = torch.from_numpy(lens.astype(np.int32)).to("cuda")
    tk.fill_synthetic_blocks(data, d_off, d_len)
    ref = tk.crc32_batch(data, d_off, d_len).clone()
    out = torch.empty_like(ref)
    lib.explore_irr_name.restype = ctypes.c_char_p
    lib.explore_run_irr.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_void_p,
                                                                              ctypes.c_void_p]
    names = [lib.explore_irr_name(i).decode() for i in range(lib.explore_irr_count())]
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    args = lambda i: (i, ctypes.c_void_p(data.data_ptr()), ctypes.c_void_p(d_off.data_ptr()),
                      ctypes.c_void_p(d_len.data_ptr()), lens.size, ctypes.c_void_p(out.data_ptr()), sp)
    sel = [i for i in range(len(names)) if not a.only or names[i] in a.only.split(",")]
    res = {i: [] for i in sel}
    for r in range(a.rounds):
        for i in sel:
            out.zero_()
            assert lib.explore_run_irr(*args(i)) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.reps):
                lib.explore_run_irr(*args(i))
            e1.record(st)
            torch.cuda.synchronize()
            res[i].append(total / (e0.elapsed_time(e1) / a.reps) / 1e6)
            if r == 0 and not torch.equal(out, ref):
                print(f"MISMATCH {names[i]}", flush=True)
    for i in sel:
        v = np.array(res[i])
        print(f"{names[i]:22s} median {np.median(v):8.1f} GB/s  min {v.min():8.1f}  max {v.max():8.1f}  "
              f"({np.median(v) / 8000 * 100:5.1f}% of 8 TB/s)", flush=True)
    sys.exit(0)
n = int(a.gib * (1 << 30)) // a.len
data = torch.empty(n * a.len, dtype=torch.uint8, device="cuda")
tk.fill_synthetic_uniform(data, a.len, n)
if a.zero:
    data.zero_()
ref = tk.crc32_batch_uniform(data, a.len, n).clone()
out = torch.empty(n, dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream()
sp = ctypes.c_void_p(st.cuda_stream)
res = {i: [] for i in sel}
for r in range(a.rounds):
    for i in sel:
        out.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        assert lib.explore_run(i, ctypes.c_void_p(data.data_ptr()), n, a.len, ctypes.c_void_p(out.data_ptr()), sp) == 0
        e0.record(st)
        for _ in range(a.reps):
            lib.explore_run(i, ctypes.c_void_p(data.data_ptr()), n, a.len, ctypes.c_void_p(out.data_ptr()), sp)
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        res[i].append(n * a.len / ms / 1e6)
        if r == 0 and names[i].startswith(("crc", "packed", "dyn", "xq")):
            ok = torch.equal(out, ref)
            if not ok:
                print(f"MISMATCH {names[i]}", flush=True)
for i in sel:
    v = np.array(res[i])
    print(f"{names[i]:22s} median {np.median(v):8.1f} GB/s  min {v.min():8.1f}  max {v.max():8.1f}  "
          f"({np.median(v) / 8000 * 100:5.1f}% of 8 TB/s)", flush=True)
