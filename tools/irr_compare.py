#!/usr/bin/env python3
"""Same cfg4 buffer, same process: product tkv_crc32_batch_device vs the explorer's T768 D4 I2
irregular variant, interleaved (explains a bench-vs-explorer gap)."""
import ctypes, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import tinykvpp_amd as tk
from conftest import Oracle
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libexplore.so"))
lib.explore_irr_name.restype = ctypes.c_char_p
lib.explore_run_irr.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
names = [lib.explore_irr_name(i).decode() for i in range(lib.explore_irr_count())]
vi = names.index("irr T768 D4 I2")
torch.cuda.set_device(0); tk.set_device(0)
ora = Oracle(os.path.join(ROOT, "oracle", "liboracle.so"))
lens = ora.zipf_lengths(1, 0, 1 << 17)
offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
total = int(lens.sum())
data = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
d_off = torch.from_numpy(offs).to("cuda"); d_len = torch.from_numpy(lens.astype(np.int32)).to("cuda")
tk.fill_synthetic_blocks(data, d_off, d_len)
out = torch.empty(lens.size, dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream(); sp = ctypes.c_void_p(st.cuda_stream)
def prod(): tk.crc32_batch(data, d_off, d_len, out=out, stream=st)
def expl(): lib.explore_run_irr(vi, ctypes.c_void_p(data.data_ptr()), ctypes.c_void_p(d_off.data_ptr()),
                                ctypes.c_void_p(d_len.data_ptr()), lens.size, ctypes.c_void_p(out.data_ptr()), sp)
def timeit(f, reps=10):
    f(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps): f()
    e1.record(st); torch.cuda.synchronize()
    return total / (e0.elapsed_time(e1) / reps) / 1e6
for r in range(4):
    print(f"round {r}: product {timeit(prod):8.1f} GB/s   explorer {timeit(expl):8.1f} GB/s", flush=True)
