"""Run a script against another build of libtkv_crc32.so (A/B of two builds on one box, one call).

    python tools/ab_lib.py path/to/libtkv_crc32.so bench.py --config cfg4 ...

Preloads the given library into tinykvpp_amd's ctypes cache, then runs the script as __main__.
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (torch's HIP runtime first, as in every product process)
import tinykvpp_amd._lib as L  # noqa: E402

lib, script = os.path.abspath(sys.argv[1]), sys.argv[2]
L.load_library(path=lib)
sys.argv = [script] + sys.argv[3:]
runpy.run_path(script, run_name="__main__")
