#!/usr/bin/env python3
"""Speculative WAL walk through LDS (tools/walk_probe.hip) against the product's device WAL verify on the
same 1 GiB image of small records (not product code). Checks the probe's per-piece starts and record
slots against the true record offsets.

    python tools/walk_probe.py [--rounds 5]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tinykvpp_amd as tk  # noqa: E402

VP, U64, U32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    tk.set_device(0)
    lib = tk.load_library()
    pl = ctypes.CDLL(os.path.join(ROOT, "tools", "ab", "libwalk_probe.so"))
    pl.walk_probe.argtypes = [VP, U64, VP, VP, VP, VP, ctypes.c_int, ctypes.c_int, VP]
    pl.walk_probe_slots.restype = U32
    pl.walk_probe_piece.restype = U32
    SL, P = pl.walk_probe_slots(), pl.walk_probe_piece()
    rng = np.random.default_rng(1)
    n = 18_199_191
    klen = rng.integers(4, 24, n).astype(np.uint64)
    vlen = rng.integers(0, 40, n).astype(np.uint64)
    size = 26 + klen + vlen
    offs = np.concatenate([[0], np.cumsum(size[:-1], dtype=np.uint64)]).astype(np.uint64)
    w = rng.integers(0, 256, int(size.sum()), dtype=np.uint8)
    for col, vals in ((0, size - 8), (18, klen), (22, vlen)):
        for b in range(4):
            w[offs.astype(np.int64) + col + b] = ((vals >> (8 * b)) & 0xFF).astype(np.uint8)
    for col in (8, 17):
        w[offs.astype(np.int64) + col] = 0
    s32 = size.astype(np.uint32)
    tk.check(lib.tkv_wal_stamp(VP(w.ctypes.data), VP(offs.ctypes.data), VP(s32.ctypes.data), n))
    total = w.size
    d = torch.from_numpy(w).cuda()
    K = (total + P - 1) // P
    S = torch.empty(K, dtype=torch.int32, device="cuda")
    X = torch.empty(K, dtype=torch.int32, device="cuda")
    C = torch.empty(K, dtype=torch.int32, device="cuda")
    slots = torch.zeros(K * SL, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    sp = VP(st.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    shapes = [(1, 9), (1, 8), (2, 4), (4, 2)]
    res = {}

    def walk(shape):
        return pl.walk_probe(VP(d.data_ptr()), total, VP(S.data_ptr()), VP(X.data_ptr()), VP(C.data_ptr()),
                             VP(slots.data_ptr()), shape[0], shape[1], sp)

    good, stop = ctypes.c_uint64(0), ctypes.c_uint64(0)

    def verify():
        return lib.tkv_wal_verify_device(VP(d.data_ptr()), total, ctypes.byref(good), ctypes.byref(stop), sp)

    for r in range(args.rounds):
        for shape in shapes:
            walk(shape)
            torch.cuda.synchronize()
            e0.record(st)
            for _ in range(args.reps):
                assert walk(shape) == 0
            e1.record(st)
            torch.cuda.synchronize()
            res.setdefault(str(shape), []).append(e0.elapsed_time(e1) / args.reps)
        verify()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            assert verify() == 0
        res.setdefault("product tkv_wal_verify_device (wall)", []).append((time.perf_counter() - t0) * 1e3 / args.reps)
    for k, v in res.items():
        print(json.dumps({"what": k, "ms": round(float(np.median(v)), 4), "GBps": round(total / np.median(v) / 1e6, 1)}),
              flush=True)
    # correctness of the last walk: each piece's start = the first true record start in it
    Sh = S.cpu().numpy().view(np.uint32)
    Ch = C.cpu().numpy().view(np.uint32)
    piece = (offs // P).astype(np.int64)
    first_in = np.full(K, 0xFFFFFFFF, np.uint64)
    idx = np.flatnonzero(np.concatenate([[True], piece[1:] != piece[:-1]]))
    first_in[piece[idx]] = offs[idx]
    has = first_in != 0xFFFFFFFF
    spec_ok = int(np.count_nonzero(Sh[has] == first_in[has].astype(np.uint32)))
    cnt_true = np.bincount(piece, minlength=K)
    cnt_ok = int(np.count_nonzero((Ch & 0x7FFFFFFF) == cnt_true))
    sl = slots.cpu().numpy().view(np.uint32).reshape(K, SL)
    rank = np.arange(n) - idx[np.searchsorted(idx, np.arange(n), side="right") - 1]
    slot_ok = int(np.count_nonzero(sl[piece, np.minimum(rank, SL - 1)] == offs.astype(np.uint32)))
    print(json.dumps({"pieces": K, "pieces_with_records": int(has.sum()), "spec_start_right": spec_ok,
                      "count_right": cnt_ok, "records": n, "slot_right": slot_ok,
                      "verify": [good.value, stop.value, total]}), flush=True)


if __name__ == "__main__":
    main()
