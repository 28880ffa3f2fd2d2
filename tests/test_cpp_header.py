"""The reference-shaped C++ header (include/frankie_crc32.hpp) compiles with the reference's usage
patterns (CPU), and its tests pass on the GPU."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "test_frankie_crc32.cpp")
LIBDIR = os.path.join(ROOT, "tinykvpp_amd")


def build(tmp_path, host_max=None):
    exe = str(tmp_path / "test_frankie_crc32")
    flags = [] if host_max is None else [f"-DTKV_DROPIN_HOST_MAX={host_max}"]
    subprocess.run(["g++", "-std=c++20", "-O2", "-Wall", "-Wextra", "-Werror", "-Wconversion", *flags,
                    "-I", os.path.join(ROOT, "include"), SRC, "-L", LIBDIR, "-ltkv_crc32",
                    f"-Wl,-rpath,{LIBDIR}", "-o", exe], check=True)
    return exe


def test_header_compiles_and_links(tmp_path):
    assert os.path.exists(build(tmp_path))


@pytest.mark.gpu
def test_header_parity_on_gpu(tmp_path):
    """Every span through the GPU (TKV_DROPIN_HOST_MAX=0): the header's arithmetic on the device."""
    r = subprocess.run([build(tmp_path, host_max=0)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    assert "ALL PASSED" in r.stdout
