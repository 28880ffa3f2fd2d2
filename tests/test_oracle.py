"""The oracle (oracle/crc32_oracle.c) pinned against the reference's own vectors (CPU only).

Vectors: test/crc32_test.cpp:81-124 known answers, WAL records laid out per src/engine/wal.cpp,
prefixes of a synthetic block, and the SURVEY §8c/§8d synthetic-batch goldens — all produced by the
reference's compiled crc32.cpp (tests/golden/make_golden.py) and cross-checked with zlib.
"""
import struct
import zlib

import numpy as np
import pytest

from conftest import golden


def test_table_matches_reference_generator(oracle):
    k = golden("kat.json")
    t = np.zeros(256, np.uint32)
    oracle.lib.oracle_table(t.ctypes.data)
    assert [int(x) for x in t] == k["table"]
    for idx, val in k["table_checks"].items():  # crc32_test.cpp:83-87
        assert int(t[int(idx)]) == val


def test_known_answers(oracle):
    k = golden("kat.json")
    for s in k["strings"]:
        assert oracle.crc(s["text"].encode()) == s["crc"]
    assert oracle.crc(b"") == 0x00000000          # crc32_test.cpp:90-94
    assert oracle.crc(b"123456789") == 0xCBF43926  # crc32_test.cpp:96-101
    assert oracle.crc(b"The quick brown fox jumps over the lazy dog") == 0x414FA339


def test_incremental_equals_single(oracle):
    k = golden("kat.json")["incremental"]  # crc32_test.cpp:110-124
    data = k["text"].encode()
    raw = 0xFFFFFFFF
    prev = 0
    for c in k["cuts"] + [len(data)]:
        raw = oracle.update(raw, data[prev:c])
        prev = c
    assert raw ^ 0xFFFFFFFF == k["crc"] == oracle.crc(data)


def test_wal_records(oracle):
    for r in golden("wal.json")["records"]:
        rec = bytes.fromhex(r["hex"])
        record_len, crc = struct.unpack_from("<II", rec, 0)
        assert record_len == len(rec) - 8                    # wal.cpp:30-31
        assert crc == r["crc"] == oracle.crc(rec[8:])         # wal.cpp:54-58, wal_test.cpp:96-118


def test_odd_prefixes(oracle):
    g = golden("odd.json")
    buf = oracle.fill(g["seed"], g["block"], 0, 1 << 20)
    for p in g["prefixes"]:
        assert oracle.crc(buf[:p["len"]].tobytes()) == p["crc"], p["len"]


def test_synthetic_first_blocks(oracle):
    s = golden("synthetic.json")
    for cfg in ("cfg2", "cfg3"):
        c = s[cfg]
        got = oracle.synthetic(1, 0, len(c["first"]), c["len"])
        assert [int(x) for x in got] == c["first"]
        assert int(oracle.synthetic(1, c["nblocks"] - 1, 1, c["len"])[0]) == c["last"]


def test_zipf_generator(oracle):
    c = golden("synthetic.json")["cfg4"]
    lens = oracle.zipf_lengths(1, 0, c["nblocks"])
    assert [int(x) for x in lens[:len(c["first_lens"])]] == c["first_lens"]
    assert int(lens.sum()) == c["total_bytes"] == 5464418334
    assert int(lens.min()) >= 256 and int(lens.max()) <= 1 << 20
    got = oracle.synthetic_lens(1, 0, lens[:64])
    assert [int(x) for x in got] == c["first"][:64]


def test_against_zlib_random(oracle):
    rng = np.random.default_rng(7)
    for n in list(range(0, 70)) + [255, 256, 1000, 4095, 4096, 4097, 65537]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert oracle.crc(d) == zlib.crc32(d)


def test_against_compiled_reference(oracle, ref_lib):
    rng = np.random.default_rng(11)
    for n in [0, 1, 3, 4, 5, 63, 64, 65, 4096, 12345]:
        d = rng.integers(0, 256, n, dtype=np.uint8)
        assert ref_lib.ref_crc32(d.ctypes.data if n else None, n) == oracle.crc(d.tobytes())


@pytest.mark.parametrize("n", [0, 1, 2, 3, 4, 7, 100])
def test_init_identity(oracle, n):
    """crc_s(D) = Shift_|D|(s) ^ crc_0(D): the identity the kernel uses to inject the init."""
    rng = np.random.default_rng(n)
    d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    for s in [0xFFFFFFFF, 0x12345678, 0]:
        shifted = oracle.update(s, b"\0" * n)
        assert oracle.update(s, d) == shifted ^ oracle.update(0, d)
