#!/usr/bin/env python3
"""Small uniform blocks (not product code): a batch of n blocks of L < 4 KiB bytes back to back,
through the uniform entry point and through the irregular one (explicit offsets and lengths), in one
process. GB/s of payload over HIP events around K launches on one stream; results must agree."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tinykvpp_amd as tk  # noqa: E402

torch.cuda.set_device(0)
tk.set_device(0)
total = 1 << 30
buf = torch.empty(total + 4096, dtype=torch.uint8, device="cuda")
tk.fill_synthetic_uniform(buf, 4096, (total + 4096) // 4096)
for L in [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else "36,64,128,512,1024,2048,3000,4095".split(","))]:
    n = total // L
    offs = torch.arange(n, dtype=torch.int64, device="cuda") * L
    lens = torch.full((n,), L, dtype=torch.int32, device="cuda")
    out_u = torch.empty(n, dtype=torch.int32, device="cuda")
    out_i = torch.empty(n, dtype=torch.int32, device="cuda")
    res = {}
    for name, fn in (("uniform", lambda: tk.crc32_batch_uniform(buf, L, n, out=out_u)),
                     ("irregular", lambda: tk.crc32_batch(buf, offs, lens, out=out_i))):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        K = 10
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(K):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = n * L * K / (e0.elapsed_time(e1) * 1e-3) / 1e9
    same = torch.equal(out_u, out_i)
    print(f"L={L:5d} n={n:9d} uniform {res['uniform']:7.1f} GB/s  irregular {res['irregular']:7.1f} GB/s  same={same}",
          flush=True)
