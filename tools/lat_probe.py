#!/usr/bin/env python3
"""Per-call latency of tkv_crc32_update (the drop-in per-record path) on host spans of several sizes."""
import ctypes, json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import tinykvpp_amd as tk  # noqa: E402
from conftest import Oracle  # noqa: E402
tk.set_device(0)
lib = tk.load_library()
ora = Oracle(os.path.join(ROOT, "oracle", "liboracle.so"))
rng = np.random.default_rng(3)
res = ctypes.c_uint32()
for nbytes in (36, 4096, 65536, 262144, 262145, 1 << 20, 16 << 20):
    payload = rng.integers(0, 256, nbytes, dtype=np.uint8)
    call = lambda: tk.check(lib.tkv_crc32_update(0xFFFFFFFF, ctypes.c_void_p(payload.ctypes.data), nbytes,
                                                 ctypes.byref(res)))
    call()
    ts = []
    for _ in range(30):
        t0 = time.perf_counter(); call(); ts.append(time.perf_counter() - t0)
    ok = (res.value ^ 0xFFFFFFFF) == ora.crc(payload.tobytes())
    print(json.dumps({"bytes": nbytes, "us_median": round(float(np.median(ts)) * 1e6, 1),
                      "us_min": round(min(ts) * 1e6, 1), "bit_exact": ok}), flush=True)
