#!/usr/bin/env python3
"""PCIe probe (not product): how fast do host bytes reach the CRC engine?

  copy  : hipMemcpyAsync pinned host -> HBM (copy engines), 1..4 streams in parallel
  mapped: the packed CRC kernel reading the pinned host buffer directly (zero copy, one pass)

Prints one line per mode with GB/s over the same pinned 4 GiB buffer of 64 KiB blocks."""
import argparse
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tinykvpp_amd as tk  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--gib", type=float, default=4.0)
ap.add_argument("--len", type=int, default=65536)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()

torch.cuda.set_device(0)
tk.set_device(0)
lib = tk.load_library()
n = int(a.gib * (1 << 30)) // a.len
total = n * a.len
dev = torch.empty(total, dtype=torch.uint8, device="cuda")
tk.fill_synthetic_uniform(dev, a.len, n)
want = tk.crc32_batch_uniform(dev, a.len, n).clone()
host = torch.empty(total, dtype=torch.uint8).pin_memory()
host.copy_(dev)
torch.cuda.synchronize()


def timed(fn):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / a.reps


for ns in (1, 2, 4):
    streams = [torch.cuda.Stream() for _ in range(ns)]
    step = total // ns

    def copy():
        for i, s in enumerate(streams):
            with torch.cuda.stream(s):
                dev[i * step:(i + 1) * step].copy_(host[i * step:(i + 1) * step], non_blocking=True)

    dt = timed(copy)
    print(f"copy   streams={ns}  {total / dt / 1e9:7.2f} GB/s", flush=True)

out = torch.empty(n, dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream()
fn = lib.tkv_crc32_batch_uniform_device
fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
               ctypes.c_void_p]


def mapped():
    rc = fn(ctypes.c_void_p(host.data_ptr()), a.len, a.len, None, ctypes.c_void_p(out.data_ptr()), n,
            ctypes.c_void_p(st.cuda_stream))
    assert rc == 0, rc


dt = timed(mapped)
ok = torch.equal(out, want)
print(f"mapped packed kernel  {total / dt / 1e9:7.2f} GB/s  bit_exact={ok}", flush=True)
