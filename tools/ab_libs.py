#!/usr/bin/env python3
"""In-process A/B of two builds of libtkv_crc32.so on the same device buffers (not product code).

    python tools/ab_libs.py tools/ab/libtkv_old.so tinykvpp_amd/libtkv_crc32.so [--rounds 6]

Both libraries are loaded side by side (separate ctypes handles, separate HIP modules). For each
workload the two builds run K launches each, interleaved round by round, on one stream; every
result array is compared between the builds. Prints one JSON line per workload with the per-round
GB/s of each build and the median ratio B/A.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import Oracle  # noqa: E402

VP = ctypes.c_void_p
U64 = ctypes.c_uint64


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path))
    lib.tkv_crc32_batch_uniform_device.argtypes = [VP, U64, U64, VP, VP, U64, VP]
    lib.tkv_crc32_batch_device.argtypes = [VP, VP, VP, VP, VP, U64, VP]
    lib.tkv_fill_synthetic_uniform.argtypes = [VP, U64, U64, U64, U64, U64, VP]
    lib.tkv_fill_synthetic_blocks.argtypes = [VP, VP, VP, U64, U64, U64, VP]
    assert lib.tkv_set_device(0) == 0
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib_a")
    ap.add_argument("lib_b")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--only", default=None, help="run only workloads whose name contains this")
    ap.add_argument("--no-check", action="store_true", help="timing probes of builds known to differ")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    A, B = load(args.lib_a), load(args.lib_b)
    st = torch.cuda.current_stream()
    sp = VP(st.cuda_stream)

    ora = Oracle(os.path.join(ROOT, "oracle", "liboracle.so"))
    lens = ora.zipf_lengths(1, 0, 1 << 17)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
    zipf_total = int(lens.sum())
    cap = max(4 << 30, zipf_total + 64)
    data = torch.empty(cap, dtype=torch.uint8, device="cuda")
    d_off = torch.from_numpy(offs).to("cuda")
    d_len = torch.from_numpy(lens.astype(np.int32)).to("cuda")
    outs = {k: torch.empty(1 << 20, dtype=torch.int32, device="cuda") for k in "AB"}

    def uniform(lib, out, blen, n):
        return lambda: lib.tkv_crc32_batch_uniform_device(VP(data.data_ptr()), blen, blen, None,
                                                          VP(out.data_ptr()), n, sp)

    def irregular(lib, out):
        return lambda: lib.tkv_crc32_batch_device(VP(data.data_ptr()), VP(d_off.data_ptr()), VP(d_len.data_ptr()),
                                                  None, VP(out.data_ptr()), lens.size, sp)

    n64 = 1 << 16
    d_off64 = torch.arange(n64, dtype=torch.int64, device="cuda") * 65536
    d_len64 = torch.full((n64,), 65536, dtype=torch.int32, device="cuda")

    def irregular64(lib, out):
        return lambda: lib.tkv_crc32_batch_device(VP(data.data_ptr()), VP(d_off64.data_ptr()), VP(d_len64.data_ptr()),
                                                  None, VP(out.data_ptr()), n64, sp)

    work = [
        ("cfg2 1M x 4 KiB", 4096, 1 << 20),
        ("64K x 64 KiB", 65536, 1 << 16),
        ("cfg4 Zipf 128K", None, lens.size),
        ("64K x 64 KiB via irregular API", -65536, n64),
    ]
    for name, blen, n in work:
        if args.only and args.only not in name:
            continue
        if blen and blen < 0:
            A.tkv_fill_synthetic_uniform(VP(data.data_ptr()), -blen, -blen, 0, n, 1, sp)
            fa, fb = irregular64(A, outs["A"]), irregular64(B, outs["B"])
            nbytes = -blen * n
        elif blen:
            A.tkv_fill_synthetic_uniform(VP(data.data_ptr()), blen, blen, 0, n, 1, sp)
            fa, fb = uniform(A, outs["A"], blen, n), uniform(B, outs["B"], blen, n)
            nbytes = blen * n
        else:
            A.tkv_fill_synthetic_blocks(VP(data.data_ptr() ), VP(d_off.data_ptr()), VP(d_len.data_ptr()), 0,
                                        lens.size, 1, sp)
            fa, fb = irregular(A, outs["A"]), irregular(B, outs["B"])
            nbytes = zipf_total
        ga, gb = [], []
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

        def run(f):
            for _ in range(10):
                assert f() == 0
            e0.record(st)
            for _ in range(args.reps):
                f()
            e1.record(st)
            torch.cuda.synchronize()
            return nbytes * args.reps / (e0.elapsed_time(e1) * 1e6)

        for r in range(args.rounds):
            if r % 2 == 0:
                ga.append(run(fa)); gb.append(run(fb))
            else:
                gb.append(run(fb)); ga.append(run(fa))
        same = bool(torch.equal(outs["A"][:n], outs["B"][:n])) or args.no_check
        print(json.dumps({"workload": name, "a_GBps": [round(x, 1) for x in ga], "b_GBps": [round(x, 1) for x in gb],
                          "median_b_over_a": round(float(np.median(np.array(gb) / np.array(ga))), 4),
                          "results_identical": same}), flush=True)
        assert same


if __name__ == "__main__":
    main()
