#!/usr/bin/env python3
"""Where inside one launch of the packed kernel the bandwidth goes: per-wave progress stamps
(s_memrealtime, 100 MHz) every 16 rows (4 KiB blocks) or 64 rows (64 KiB blocks), turned into the
chip-wide completion rate per 20 us bin, for a launch run back to back on one stream and for one run
alternating with another stream (tools/overlap_probe.py's two modes)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tinykvpp_amd as tk  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libexplore.so"))
lib.explore_prog.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p]
torch.cuda.set_device(0)
tk.set_device(0)
blen = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
PROG = 16 if blen == 4096 else 64
n = (4 << 30) // blen
data = torch.empty(n * blen, dtype=torch.uint8, device="cuda")
tk.fill_synthetic_uniform(data, blen, n)
ref = tk.crc32_batch_uniform(data, blen, n).clone()
W = torch.cuda.get_device_properties(0).multi_processor_count * 16
SLOTS = 64
K = 8
stamps = [torch.zeros(W * SLOTS, dtype=torch.int64, device="cuda") for _ in range(K)]
outs = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(2)]
s0 = torch.cuda.current_stream()
s1 = torch.cuda.Stream()
rows_per_wave = n * (blen // 4096) // W


def run(two):
    for st in stamps:
        st.zero_()
    torch.cuda.synchronize()
    s1.wait_stream(s0)
    for i in range(K):
        s = s1 if (two and i % 2) else s0
        assert lib.explore_prog(ctypes.c_void_p(data.data_ptr()), n, blen, ctypes.c_void_p(outs[i % 2].data_ptr()),
                                ctypes.c_void_p(stamps[i].data_ptr()), ctypes.c_void_p(s.cuda_stream)) == 0
    s0.wait_stream(s1)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], ref) and torch.equal(outs[1], ref)
    return [st.cpu().numpy().reshape(W, SLOTS).astype(np.float64) * 10.0 for st in stamps]  # ns


def curve(S, t0):
    """(completion times, rows) events of one launch: PROG rows complete at every stamp after the first
    row stamp; the end stamp closes the last group."""
    ts, rows = [], []
    nst = 1 + (rows_per_wave + PROG - 1) // PROG  # row stamps 1..nst-1, end stamp nst
    for w in range(W):
        for s in range(2, nst + 1):
            ts.append(S[w, s] - t0)
            rows.append(min(PROG, rows_per_wave - (s - 2) * PROG))
    return np.array(ts), np.array(rows)


for r in range(2):
    for two in (False, True):
        res = run(two)
        i = K // 2  # a launch from the middle of the sequence
        S = res[i]
        t0 = S[:, 0].min()
        tend = S.max() - t0
        ts, rows = curve(S, t0)
        bins = np.arange(0, tend + 20e3, 20e3)
        h, _ = np.histogram(ts, bins=bins, weights=rows * 4096.0)
        gbs = h / 20e3  # bytes per ns = GB/s
        fill = np.median(S[:, 1] - S[:, 0]) / 1e3
        first = (S[:, 1] - t0).max() / 1e3
        ends = (S.max(axis=1) - t0) / 1e3
        print(f"{'two streams' if two else 'one stream '} launch {i}: span {tend/1e3:.1f} us, table fill "
              f"median {fill:.2f} us (last wave past it at {first:.1f} us), wave end p10/p50/p90/max "
              f"{np.percentile(ends,10):.0f}/{np.percentile(ends,50):.0f}/{np.percentile(ends,90):.0f}/{ends.max():.0f} us",
              flush=True)
        print("   GB/s per 20 us bin: " + " ".join(f"{g:.0f}" for g in gbs), flush=True)
        if two:
            # the neighbouring launches (other stream) overlap this one's ends
            P, N = res[i - 1], res[i + 1]
            print(f"   previous launch ends {(P.max() - t0)/1e3:.1f} us, next launch starts {(N[:, 0].min() - t0)/1e3:.1f} us",
                  flush=True)
        else:
            P = res[i - 1]
            print(f"   gap after previous launch: {(t0 - P.max())/1e3:.1f} us", flush=True)
