#!/usr/bin/env python3
"""Launch-boundary probe: the cfg2 batch (1 M x 4 KiB) checksummed back to back on ONE stream (the
bench's shape) vs the same launches alternating between TWO streams, so that a launch's workgroups
can take the CUs its predecessor frees while that one's slowest waves finish. The gap between the
two rates is what the kernel loses at its ends (ramp-up and wave tail)."""
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
n = (4 << 30) // blen
data = torch.empty(n * blen, dtype=torch.uint8, device="cuda")
tk.fill_synthetic_uniform(data, blen, n)
outs = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(2)]
s0 = torch.cuda.current_stream()
s1 = torch.cuda.Stream()
K = 40
for _ in range(50):
    tk.crc32_batch_uniform(data, blen, n, out=outs[0], stream=s0)
torch.cuda.synchronize()
res = {"one stream": [], "two streams": []}
for r in range(6):
    for mode in res:
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record(s0)
        s1.wait_stream(s0)
        for i in range(K):
            s = s1 if (mode == "two streams" and i % 2) else s0
            tk.crc32_batch_uniform(data, blen, n, out=outs[i % 2], stream=s)
        s0.wait_stream(s1)
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record(s0)
        torch.cuda.synchronize()
        res[mode].append(K * n * blen / (e0.elapsed_time(e1) * 1e-3) / 1e9)
for mode, v in res.items():
    v = np.array(v)
    print(f"{mode:12s} median {np.median(v):7.1f} GB/s  min {v.min():7.1f}  max {v.max():7.1f}  "
          f"({np.median(v) / 8000 * 100:4.1f}% of 8 TB/s)", flush=True)
assert torch.equal(outs[0], outs[1])
