#!/usr/bin/env python3
"""End-to-end host-memory rate (SURVEY §8d cfg3 "+ H2D/D2H timed"): blocks start in (pinned or
pageable) host memory, results end in host memory; tkv_crc32_batch_host streams them through the
GPU (H2D copy, kernel, D2H results overlapped on two streams). Prints one JSON line per mode."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tinykvpp_amd as tk  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--len", type=int, default=65536)
ap.add_argument("--gib", type=float, default=16.0)
ap.add_argument("--steps", type=int, default=3)
a = ap.parse_args()

torch.cuda.set_device(0)
tk.set_device(0)
n = int(a.gib * (1 << 30)) // a.len
total = n * a.len
# generate on the device in 4 GiB pieces, copy into pinned host memory
host_t = torch.empty(total, dtype=torch.uint8).pin_memory()
piece = (4 << 30) // a.len
dev = torch.empty(piece * a.len, dtype=torch.uint8, device="cuda")
want = np.zeros(n, np.uint32)
for b0 in range(0, n, piece):
    m = min(piece, n - b0)
    tk.fill_synthetic_uniform(dev, a.len, m, first_block=b0)
    want[b0:b0 + m] = tk.crc32_batch_uniform(dev, a.len, m).cpu().numpy().view(np.uint32)
    host_t[b0 * a.len:(b0 + m) * a.len].copy_(dev[:m * a.len])
del dev
torch.cuda.synchronize()
host = host_t.numpy()
offs = np.arange(n, dtype=np.uint64) * a.len
lens = np.full(n, a.len, np.uint32)

lib = tk.load_library()
for mode in ("pinned", "pinned-staged", "pageable"):
    lib.tkv_debug_set_host_mapped(0 if mode == "pinned-staged" else 1)  # zero copy vs staged copies
    src = host if mode.startswith("pinned") else np.array(host[: min(total, 4 << 30)])
    nn = src.size // a.len
    got = tk.crc32_batch_host(src, offs[:nn], lens[:nn])  # warm-up + correctness
    ok = bool(np.array_equal(got, want[:nn]))
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tk.crc32_batch_host(src, offs[:nn], lens[:nn])
    dt = (time.perf_counter() - t0) / a.steps
    print(json.dumps({"mode": f"e2e host ({mode}) -> GPU -> host", "blocks": nn, "block_bytes": a.len,
                      "bytes": nn * a.len, "seconds": round(dt, 4),
                      "GiB_per_s": round(nn * a.len / (1 << 30) / dt, 2),
                      "GB_per_s": round(nn * a.len / 1e9 / dt, 2), "bit_exact": ok}), flush=True)
