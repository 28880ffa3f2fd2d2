#!/usr/bin/env python3
"""tkv_wal_stamp over 400 K pageable records (430 MB), five times: a short program for a trace of
where a large group-commit stamp spends its time (not product code)."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VP, U64 = ctypes.c_void_p, ctypes.c_uint64
lib = ctypes.CDLL(os.path.join(ROOT, "tinykvpp_amd", "libtkv_crc32.so"))
lib.tkv_wal_stamp.argtypes = [VP, VP, VP, U64]
assert lib.tkv_set_device(0) == 0
rng = np.random.default_rng(1)
n = 400_000
klen = rng.integers(8, 64, n).astype(np.uint32)
vlen = np.minimum(rng.zipf(1.6, n) * 64, 16_000).astype(np.uint32)
size = (26 + klen + vlen).astype(np.uint32)
offs = np.concatenate([[0], np.cumsum(size[:-1], dtype=np.uint64)]).astype(np.uint64)
wal = rng.integers(0, 256, int(size.sum()), dtype=np.uint8)
for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    t0 = time.perf_counter()
    assert lib.tkv_wal_stamp(VP(wal.ctypes.data), VP(offs.ctypes.data), VP(size.ctypes.data), n) == 0
    print(f"stamp {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
