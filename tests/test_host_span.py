"""The opt-in host latency path for one short span (tkv_crc32[c]_update_host, include/tkv_crc32.h;
the drop-in header routes spans of at most TKV_DROPIN_HOST_MAX bytes there when an integrator
defines it). Product code, so it is pinned like every other path: the reference's known answers
(test/crc32_test.cpp:81-124, tests/golden/kat.json), the reference's CRC of the WAL records of
test/wal_test.cpp (tests/golden/wal.json), the prefixes of a synthetic block (odd.json), RFC 3720
vectors for CRC-32C, and the oracle on random spans. No GPU is involved."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, golden
from test_oracle import RFC3720_B4


@pytest.fixture(scope="module")
def span(lib):
    for name in ("tkv_crc32_update_host", "tkv_crc32c_update_host"):
        f = getattr(lib, name)
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32)]

    def run(raw, data, algo="crc32"):
        a = np.frombuffer(bytes(data), np.uint8)
        out = ctypes.c_uint32(0)
        rc = getattr(lib, f"tkv_{algo}_update_host")(raw, a.ctypes.data if a.size else None, a.size,
                                                       ctypes.byref(out))
        assert rc == 0
        return out.value
    return run


def test_known_answers(span):
    kat = golden("kat.json")
    for s in kat["strings"]:
        assert span(0xFFFFFFFF, s["text"].encode()) ^ 0xFFFFFFFF == s["crc"], s["text"]
    inc = kat["incremental"]
    text, (c1, c2) = inc["text"].encode(), inc["cuts"]
    r = 0xFFFFFFFF
    for piece in (text[:c1], text[c1:c2], text[c2:]):
        r = span(r, piece)
    assert r ^ 0xFFFFFFFF == inc["crc"]


def test_wal_records(span):
    for rec in golden("wal.json")["records"]:
        b = bytes.fromhex(rec["hex"])
        assert span(0xFFFFFFFF, b[8:]) ^ 0xFFFFFFFF == rec["crc"] == int.from_bytes(b[4:8], "little")


def test_synthetic_prefixes(span, oracle):
    g = golden("odd.json")
    longest = max(p["len"] for p in g["prefixes"])
    blk = oracle.fill(g["seed"], g["block"], 0, longest).tobytes()
    for p in g["prefixes"]:
        assert span(0xFFFFFFFF, blk[:p["len"]]) ^ 0xFFFFFFFF == p["crc"], p["len"]


def test_random_spans_and_chaining(span, oracle):
    rng = np.random.default_rng(11)
    buf = rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()
    for n in list(range(0, 70)) + [127, 128, 129, 4095, 4096, 4097, 65536]:
        off = int(rng.integers(0, 8))
        raw = int(rng.integers(0, 2**32))
        assert span(raw, buf[off:off + n]) == oracle.update(raw, buf[off:off + n]), (n, off)
    r = 0xFFFFFFFF
    cuts = np.sort(rng.integers(0, len(buf), 40))
    prev = 0
    for c in list(cuts) + [len(buf)]:
        r = span(r, buf[prev:c])
        prev = c
    assert r ^ 0xFFFFFFFF == oracle.crc(buf)


@pytest.mark.parametrize("data,want", RFC3720_B4)
def test_crc32c_vectors(span, data, want):
    assert span(0xFFFFFFFF, data, "crc32c") ^ 0xFFFFFFFF == want


def test_crc32c_random(span, oracle):
    rng = np.random.default_rng(12)
    for n in (0, 1, 7, 8, 9, 36, 1000, 5000):
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        raw = int(rng.integers(0, 2**32))
        assert span(raw, b, "crc32c") == oracle.update_c(raw, b)


def test_null_arguments(lib, span):
    out = ctypes.c_uint32(0)
    assert lib.tkv_crc32_update_host(0, None, 0, ctypes.byref(out)) == 0
    assert lib.tkv_crc32_update_host(0, None, 5, ctypes.byref(out)) == 3  # TKV_INVALID_ARGUMENT
    assert lib.tkv_crc32_update_host(0, None, 0, None) == 3


def _run_dropin(tmp_path):
    exe = str(tmp_path / "test_dropin_host_span")
    lib = os.path.join(ROOT, "tinykvpp_amd")
    subprocess.run(["g++", "-std=c++20", "-O2", "-Wall", "-Wextra", "-Werror", "-Wconversion",
                    "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "test_dropin_host_span.cpp"), "-L", lib, "-ltkv_crc32",
                    f"-Wl,-rpath,{lib}", "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    assert "ALL PASSED" in r.stdout
    return r


def test_dropin_header_host_spans_on_cpu(tmp_path):
    """The drop-in header with its default threshold (64 KiB): every span of the reference's usage
    (crc32_test.cpp known answers, chained updates, wal_entry::encode's record CRC) runs on the host,
    the per-thread counters show no GPU call, and a 36-byte put costs no more than the reference's
    byte loop on the same core. Spans above the threshold (1 MiB, a 128 KiB WAL record) try the GPU;
    on this GPU-less machine the header recomputes them on the host after the error, with one
    warning, instead of aborting: crc32::update never fails (crc32.cpp:9-16)."""
    r = _run_dropin(tmp_path)
    if "no GPU" in r.stdout:
        assert "GPU calls 3, host recomputes 3" in r.stdout
        assert r.stderr.count("recomputed on the host") == 1  # one warning per process


@pytest.mark.gpu
def test_dropin_header_on_gpu(gpu, tmp_path):
    """The same binary on the GPU box: the long spans take the GPU and nothing is recomputed."""
    r = _run_dropin(tmp_path)
    assert "GPU present; GPU calls 3, host recomputes 0" in r.stdout, r.stdout
