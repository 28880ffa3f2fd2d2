#!/usr/bin/env python3
"""In-process A/B of builds of libtkv_crc32.so on uniform small blocks (not product code): 4 GiB as
blocks of 64-2048 bytes, every library in rotation on the same buffer; results must agree.

    python tools/ab_small_uniform.py lib1.so lib2.so ... [--rounds 6]
"""
import argparse
import ctypes
import json
import os

import numpy as np
import torch

VP, U64 = ctypes.c_void_p, ctypes.c_uint64
ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+")
ap.add_argument("--rounds", type=int, default=6)
args = ap.parse_args()
torch.cuda.set_device(0)
libs = []
for p in args.libs:
    lib = ctypes.CDLL(os.path.abspath(p))
    lib.tkv_crc32_batch_uniform_device.argtypes = [VP, U64, U64, VP, VP, U64, VP]
    lib.tkv_fill_synthetic_uniform.argtypes = [VP, U64, U64, U64, U64, U64, VP]
    lib.tkv_crc32_batch_device.argtypes = [VP, VP, VP, VP, VP, U64, VP]
    assert lib.tkv_set_device(0) == 0
    libs.append(lib)
total = 4 << 30
buf = torch.empty(total, dtype=torch.uint8, device="cuda")
st = VP(torch.cuda.current_stream().cuda_stream)
assert libs[0].tkv_fill_synthetic_uniform(VP(buf.data_ptr()), 4096, 4096, 0, total // 4096, 1, st) == 0
K = 20
irregular = os.environ.get("AB_IRREGULAR") == "1"  # the same blocks through the irregular entry point
for L in [int(x) for x in os.environ.get("AB_LENS", "64,128,512,1024,2048").split(",")]:
    n = total // L
    outs = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in libs]
    if irregular:
        n = min(n, (1 << 22) - 64)  # stream mode covers up to 4 M blocks (1024 prepass tiles)
        offs = torch.arange(n, dtype=torch.int64, device="cuda") * L
        lens = torch.full((n,), L, dtype=torch.int32, device="cuda")
    times = [[] for _ in libs]
    for r in range(args.rounds):
        for i, lib in enumerate(libs):
            if irregular:
                run = lambda: lib.tkv_crc32_batch_device(VP(buf.data_ptr()), VP(offs.data_ptr()), VP(lens.data_ptr()),  # noqa: E731
                                                         None, VP(outs[i].data_ptr()), n, st)
            else:
                run = lambda: lib.tkv_crc32_batch_uniform_device(VP(buf.data_ptr()), L, L, None, VP(outs[i].data_ptr()), n, st)  # noqa: E731
            for _ in range(3):
                assert run() == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(K):
                run()
            e1.record()
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1) / K)
    for i, p in enumerate(args.libs):
        ms = float(np.median(times[i]))
        print(json.dumps({"block": L, "irregular": irregular, "blocks": n, "lib": os.path.basename(p),
                          "median_ms": round(ms, 4), "GB_per_s": round(n * L / ms / 1e6, 1),
                          "same_as_first": bool(torch.equal(outs[i][:n], outs[0][:n]))}),
              flush=True)
