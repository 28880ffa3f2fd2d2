#!/usr/bin/env python3
"""In-process comparison of several builds of libtkv_crc32.so (not product code): every library
runs every workload, rotated round by round on one stream and the same device buffers. Prints one
JSON line per (workload, library) with the median GB/s; results are checked against the first
library unless --no-check (probe builds that skip work).

    python tools/ab_multi.py lib1.so lib2.so ... [--rounds 8] [--only cfg4]
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
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--only", default=None)
    ap.add_argument("--no-check", action="store_true")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    libs = [load(p) for p in args.libs]
    st = torch.cuda.current_stream()
    sp = VP(st.cuda_stream)
    ora = Oracle(os.path.join(ROOT, "oracle", "liboracle.so"))
    lens = ora.zipf_lengths(1, 0, 1 << 17)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
    n64 = 1 << 16
    cap = max(n64 * 65536, int(lens.sum()) + 64)
    data = torch.empty(cap, dtype=torch.uint8, device="cuda")
    D = VP(data.data_ptr())
    dz_o, dz_l = torch.from_numpy(offs).to("cuda"), torch.from_numpy(lens.astype(np.int32)).to("cuda")
    dz_g = torch.from_numpy((lens - 1).astype(np.int32)).to("cuda")  # 1-byte gaps: the general walk
    d64_o = torch.arange(n64, dtype=torch.int64, device="cuda") * 65536
    d64_l = torch.full((n64,), 65536, dtype=torch.int32, device="cuda")
    outs = [torch.empty(1 << 20, dtype=torch.int32, device="cuda") for _ in libs]

    def fill_uniform():
        libs[0].tkv_fill_synthetic_uniform(D, 65536, 65536, 0, n64, 1, sp)

    def fill_zipf():
        libs[0].tkv_fill_synthetic_blocks(D, VP(dz_o.data_ptr()), VP(dz_l.data_ptr()), 0, lens.size, 1, sp)

    n4k = 1 << 20

    def fill_4k():
        libs[0].tkv_fill_synthetic_uniform(D, 4096, 4096, 0, n4k, 1, sp)

    work = [
        ("packed 1M x 4 KiB (cfg2)", fill_4k, n4k * 4096, n4k,
         lambda lib, o: lib.tkv_crc32_batch_uniform_device(D, 4096, 4096, None, o, n4k, sp)),
        ("packed 64K x 64 KiB", fill_uniform, n64 * 65536, n64,
         lambda lib, o: lib.tkv_crc32_batch_uniform_device(D, 65536, 65536, None, o, n64, sp)),
        ("stream 64K x 64 KiB", fill_uniform, n64 * 65536, n64,
         lambda lib, o: lib.tkv_crc32_batch_device(D, VP(d64_o.data_ptr()), VP(d64_l.data_ptr()), None, o, n64, sp)),
        ("cfg4 Zipf 128K", fill_zipf, int(lens.sum()), lens.size,
         lambda lib, o: lib.tkv_crc32_batch_device(D, VP(dz_o.data_ptr()), VP(dz_l.data_ptr()), None, o, lens.size,
                                                   sp)),
        ("cfg4 Zipf general (1-byte gaps)", fill_zipf, int(lens.sum()) - lens.size, lens.size,
         lambda lib, o: lib.tkv_crc32_batch_device(D, VP(dz_o.data_ptr()), VP(dz_g.data_ptr()), None, o, lens.size,
                                                   sp)),
    ]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, fill, nbytes, n, call in work:
        if args.only and args.only not in name:
            continue
        fill()
        fns = [(lambda lib=lib, o=VP(out.data_ptr()): call(lib, o)) for lib, out in zip(libs, outs)]
        g = [[] for _ in libs]
        for r in range(args.rounds):
            order = list(range(len(libs)))
            order = order[r % len(order):] + order[:r % len(order)]
            for k in order:
                for _ in range(5):
                    assert fns[k]() == 0
                e0.record(st)
                for _ in range(args.reps):
                    fns[k]()
                e1.record(st)
                torch.cuda.synchronize()
                g[k].append(nbytes * args.reps / (e0.elapsed_time(e1) * 1e6))
        for k, p in enumerate(args.libs):
            same = args.no_check or bool(torch.equal(outs[0][:n], outs[k][:n]))
            print(json.dumps({"workload": name, "lib": os.path.basename(p), "median_GBps": round(float(np.median(g[k])), 1),
                              "rel_first": round(float(np.median(np.array(g[k]) / np.array(g[0]))), 4),
                              "results_identical": same}), flush=True)


if __name__ == "__main__":
    main()
