#!/usr/bin/env python3
"""Tail-split probe: one step over the cfg2 batch as ONE launch (the bench's shape) vs the same
batch issued as a head launch of the first fraction f of the blocks on the caller's stream and a
tail launch of the rest on a side stream (forked and joined with events inside the step). The tail
launch's workgroups take the CUs the head launch's earliest workgroups free, so the spread between
CUs at the end of the head launch is filled with tail work. In-process interleaved
rounds, HIP events on the caller's stream around K steps.

usage: split_probe.py [block_bytes] [fractions comma-separated]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tinykvpp_amd as tk  # noqa: E402

torch.cuda.set_device(0)
tk.set_device(0)
blen = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
fracs = [float(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0.95, 0.9, 0.85, 0.8, 0.7]
n = (4 << 30) // blen if blen <= 4096 else (16 << 30) // blen
data = torch.empty(n * blen, dtype=torch.uint8, device="cuda")
tk.fill_synthetic_uniform(data, blen, n)
out = torch.empty(n, dtype=torch.int32, device="cuda")
s0 = torch.cuda.current_stream()
s1 = torch.cuda.Stream()
K = 40 if blen <= 4096 else 12
tk.crc32_batch_uniform(data, blen, n, out=out, stream=s0)
torch.cuda.synchronize()
ref = out.clone()


def step(f):
    if f >= 1.0:
        tk.crc32_batch_uniform(data, blen, n, out=out, stream=s0)
        return
    na = int(n * f) // 64 * 64
    s1.wait_stream(s0)
    tk.crc32_batch_uniform(data, blen, na, out=out, stream=s0)
    tk.crc32_batch_uniform(data, blen, n - na, out=out[na:], stream=s1, offset=na * blen)
    s0.wait_stream(s1)


modes = [1.0] + fracs
res = {f: [] for f in modes}
t_end = None
import time  # noqa: E402
t0 = time.time()
while time.time() - t0 < 1.5:  # warm-up floor (clock ramp)
    step(1.0)
    torch.cuda.synchronize()
for r in range(8):
    for f in modes:
        for _ in range(3):
            step(f)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s0)
        for _ in range(K):
            step(f)
        e1.record(s0)
        torch.cuda.synchronize()
        res[f].append(K * n * blen / (e0.elapsed_time(e1) * 1e-3) / 1e9)
        assert torch.equal(out, ref), f"mismatch at f={f}"
base = np.median(res[1.0])
for f, v in res.items():
    v = np.array(v)
    print(f"blen {blen} f={f:5.3f} median {np.median(v):7.1f} GB/s  min {v.min():7.1f}  max {v.max():7.1f}  "
          f"({np.median(v) / 8000 * 100:4.1f}% of 8 TB/s, {100 * (np.median(v) / base - 1):+5.2f}%)", flush=True)
