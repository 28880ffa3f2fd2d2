#!/usr/bin/env python3
"""In-process comparison of builds of libtkv_crc32.so on the host-memory batch paths (not product
code): tkv_crc32_batch_host over a pageable 430 MB WAL image's payloads, tkv_wal_stamp over the same
records, tkv_sst_stamp_blocks over a pageable 1 GB SSTable image, a pageable 4 GiB batch of
64 KiB blocks, and tkv_wal_verify of pageable WAL images (the 430 MB Zipf records, 1 GiB of small
records); libraries rotate round by round, results must agree.

    python tools/ab_host.py lib1.so lib2.so ... [--rounds 4]
"""
import argparse
import ctypes
import json
import os
import time

import numpy as np

VP, U64 = ctypes.c_void_p, ctypes.c_uint64


def wal_image(n_rec, klen, vlen, rng):
    """Records the reference encoder would write (wal.cpp:19-61), CRC fields left for tkv_wal_stamp."""
    size = 26 + klen + vlen
    offs = np.concatenate([[0], np.cumsum(size[:-1], dtype=np.uint64)]).astype(np.uint64)
    w = rng.integers(0, 256, int(size.sum()), dtype=np.uint8)
    for col, vals in ((0, size - 8), (18, klen), (22, vlen)):
        for b in range(4):
            w[offs.astype(np.int64) + col + b] = ((vals >> (8 * b)) & 0xFF).astype(np.uint8)
    for col in (8, 17):
        w[offs.astype(np.int64) + col] = 0
    return w, offs, size.astype(np.uint32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rounds", type=int, default=4)
    args = ap.parse_args()
    libs = []
    for p in args.libs:
        lib = ctypes.CDLL(os.path.abspath(p))
        lib.tkv_crc32_batch_host.argtypes = [VP, VP, VP, VP, VP, U64]
        lib.tkv_wal_stamp.argtypes = [VP, VP, VP, U64]
        lib.tkv_sst_stamp_blocks.argtypes = [VP, VP, VP, U64]
        lib.tkv_wal_verify.argtypes = [VP, U64, ctypes.POINTER(U64), ctypes.POINTER(U64)]
        assert lib.tkv_set_device(0) == 0
        libs.append(lib)
    rng = np.random.default_rng(1)
    n = 400_000
    klen = rng.integers(8, 64, n).astype(np.uint32)
    vlen = np.minimum(rng.zipf(1.6, n) * 64, 16_000).astype(np.uint32)
    size = (26 + klen + vlen).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(size[:-1], dtype=np.uint64)]).astype(np.uint64)
    wal = rng.integers(0, 256, int(size.sum()), dtype=np.uint8)
    poff, plen = offs + 8, (size - 8).astype(np.uint32)
    nblk = 250_000
    ssz = np.full(nblk, 4096, np.uint64)
    soff = np.arange(nblk, dtype=np.uint64) * 4096
    sst = rng.integers(0, 256, nblk * 4096, dtype=np.uint8)
    sst[soff.astype(np.int64)] = 20
    n64 = 65536
    big = rng.integers(0, 256, n64 * 65536, dtype=np.uint8)
    boff = np.arange(n64, dtype=np.uint64) * 65536
    blen = np.full(n64, 65536, np.uint32)
    wz, oz, sz = wal_image(n, klen, vlen, rng)
    ns = 18_199_191
    ws, os_, ss = wal_image(ns, rng.integers(4, 24, ns).astype(np.uint32), rng.integers(0, 40, ns).astype(np.uint32), rng)
    for w, o, z in ((wz, oz, sz), (ws, os_, ss)):
        assert libs[0].tkv_wal_stamp(VP(w.ctypes.data), VP(o.ctypes.data), VP(z.ctypes.data), o.size) == 0

    def verify(w):
        def call(lib, out):
            g, s_ = U64(0), U64(0)
            rc = lib.tkv_wal_verify(VP(w.ctypes.data), w.nbytes, ctypes.byref(g), ctypes.byref(s_))
            out[0], out[1] = g.value & 0xFFFFFFFF, s_.value & 0xFFFFFFFF
            return rc
        return call
    work = [
        ("batch_host WAL payloads 430 MB", wal.nbytes, lambda lib, out: lib.tkv_crc32_batch_host(
            VP(wal.ctypes.data), VP(poff.ctypes.data), VP(plen.ctypes.data), None, VP(out.ctypes.data), n), n),
        ("wal_stamp 400 K records", wal.nbytes, lambda lib, out: lib.tkv_wal_stamp(
            VP(wal.ctypes.data), VP(offs.ctypes.data), VP(size.ctypes.data), n), None),
        ("sst_stamp 250 K x 4 KiB", sst.nbytes, lambda lib, out: lib.tkv_sst_stamp_blocks(
            VP(sst.ctypes.data), VP(soff.ctypes.data), VP(ssz.ctypes.data), nblk), None),
        ("batch_host 64 K x 64 KiB (4 GiB)", big.nbytes, lambda lib, out: lib.tkv_crc32_batch_host(
            VP(big.ctypes.data), VP(boff.ctypes.data), VP(blen.ctypes.data), None, VP(out.ctypes.data), n64), n64),
        ("wal_verify Zipf 430 MB", wz.nbytes, verify(wz), 2),
        ("wal_verify small records 1 GiB", ws.nbytes, verify(ws), 2),
    ]
    for name, nbytes, call, nout in work:
        outs = [np.zeros(nout or 1, np.uint32) for _ in libs]
        times = [[] for _ in libs]
        for r in range(args.rounds + 1):
            order = list(range(len(libs)))
            order = order[r % len(order):] + order[:r % len(order)]
            for k in order:
                t0 = time.perf_counter()
                assert call(libs[k], outs[k]) == 0
                if r:
                    times[k].append(time.perf_counter() - t0)
        for k, p in enumerate(args.libs):
            med = float(np.median(times[k]))
            print(json.dumps({"work": name, "lib": os.path.basename(p), "median_ms": round(med * 1e3, 2),
                              "GB_per_s": round(nbytes / med / 1e9, 1),
                              "same_as_first": bool(np.array_equal(outs[k], outs[0]))}), flush=True)


if __name__ == "__main__":
    main()
