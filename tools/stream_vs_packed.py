#!/usr/bin/env python3
"""Profiling driver (not product code): the same 4 GiB of 64 KiB blocks through the packed kernel
(uniform API) and through stream mode (irregular API, blocks back to back), then cfg4's Zipf batch
through stream mode, `--reps` launches each, so rocprofv3 PMC passes can compare crc_packed and
crc_stream per row on identical bytes."""
import argparse
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

VP = ctypes.c_void_p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    lib = tk.load_library()
    torch.cuda.set_device(0)
    sp = VP(torch.cuda.current_stream().cuda_stream)
    n64 = 1 << 16
    ora = Oracle(os.path.join(ROOT, "oracle", "liboracle.so"))
    lens = ora.zipf_lengths(1, 0, 1 << 17)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
    cap = max(n64 * 65536, int(lens.sum()) + 64)
    data = torch.empty(cap, dtype=torch.uint8, device="cuda")
    out = torch.empty(1 << 17, dtype=torch.int32, device="cuda")
    o64 = torch.arange(n64, dtype=torch.int64, device="cuda") * 65536
    l64 = torch.full((n64,), 65536, dtype=torch.int32, device="cuda")
    oz = torch.from_numpy(offs).to("cuda")
    lz = torch.from_numpy(lens.astype(np.int32)).to("cuda")
    D, O = VP(data.data_ptr()), VP(out.data_ptr())
    lib.tkv_fill_synthetic_uniform(D, 65536, 65536, 0, n64, 1, sp)
    for _ in range(args.reps):
        assert lib.tkv_crc32_batch_uniform_device(D, 65536, 65536, None, O, n64, sp) == 0
    ref = out[:n64].clone()
    for _ in range(args.reps):
        assert lib.tkv_crc32_batch_device(D, VP(o64.data_ptr()), VP(l64.data_ptr()), None, O, n64, sp) == 0
    torch.cuda.synchronize()
    assert torch.equal(ref, out[:n64])
    lib.tkv_fill_synthetic_blocks(D, VP(oz.data_ptr()), VP(lz.data_ptr()), 0, lens.size, 1, sp)
    for _ in range(args.reps):
        assert lib.tkv_crc32_batch_device(D, VP(oz.data_ptr()), VP(lz.data_ptr()), None, O, lens.size, sp) == 0
    torch.cuda.synchronize()
    print("ok", flush=True)


if __name__ == "__main__":
    main()
