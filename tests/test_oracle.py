"""The oracle (oracle/crc32_oracle.c) pinned against the reference's own vectors (CPU only).

Vectors: test/crc32_test.cpp:81-124 known answers, WAL records laid out per src/engine/wal.cpp,
prefixes of a synthetic block, and the SURVEY §8c/§8d synthetic-batch goldens — all produced by the
reference's compiled crc32.cpp (tests/golden/make_golden.py) and cross-checked with zlib.
"""
import ctypes
import os
import struct
import sys
import zlib

import numpy as np
import pytest

from conftest import ROOT, golden


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


def test_slicing_by_8_comparison_row(oracle):
    """bench.py's 'not reference' slicing-by-8 CPU row computes the same CRC (any length, any start)."""
    lib = oracle.lib
    lib.oracle_update_s8.restype = ctypes.c_uint32
    lib.oracle_update_s8.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
    lib.oracle_crc_batch_s8.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_void_p]
    rng = np.random.default_rng(5)
    buf = rng.integers(0, 256, 70000, dtype=np.uint8)
    sizes = list(range(0, 40)) + [255, 4096, 4099, 65536]
    offs = np.array([(7 * i) % 997 for i in range(len(sizes))], np.uint64)
    lens = np.array(sizes, np.uint32)
    out = np.zeros(len(sizes), np.uint32)
    lib.oracle_crc_batch_s8(buf.ctypes.data, offs.ctypes.data, lens.ctypes.data, len(sizes), out.ctypes.data)
    for i, (o, n) in enumerate(zip(offs, lens)):
        d = buf[int(o):int(o) + int(n)].tobytes()
        assert int(out[i]) == zlib.crc32(d) == oracle.crc(d)
        assert lib.oracle_update_s8(0x12345678, buf[int(o):].ctypes.data, int(n)) == \
            oracle.lib.oracle_update(0x12345678, buf[int(o):].ctypes.data, int(n))


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


# ---- CRC-32C restatement: pinned by published vectors ----------------------

RFC3720_B4 = [  # RFC 3720 §B.4 (iSCSI CRC32C examples), values as 32-bit integers
    (bytes(32), 0x8A9136AA),
    (bytes([0xFF] * 32), 0x62A8AB43),
    (bytes(range(32)), 0x46DD794E),
    (bytes(range(31, -1, -1)), 0x113FDB5C),
    (b"123456789", 0xE3069283),  # CRC catalogue check value of CRC-32C (iSCSI)
]


@pytest.mark.parametrize("data,want", RFC3720_B4)
def test_crc32c_published_vectors(oracle, data, want):
    assert oracle.crc_c(data) == want


def test_crc32c_incremental(oracle):
    data = bytes(range(256)) * 5
    raw = 0xFFFFFFFF
    for a, b in ((0, 1), (1, 100), (100, 1280)):
        raw = oracle.update_c(raw, data[a:b])
    assert raw ^ 0xFFFFFFFF == oracle.crc_c(data)


# ---- SSTable stamp restatement (format of include/tkv_crc32.h; parity unpinned) -------------------

def test_sst_stamp_oracle_against_zlib(oracle):
    import zlib
    import tinykvpp_amd.sst as sst
    rng = np.random.default_rng(5)
    for n_entries in (1, 3, 40):
        entries = [(rng.bytes(int(rng.integers(1, 40))), rng.bytes(int(rng.integers(0, 200))))
                   for _ in range(n_entries)]
        img = bytearray(sst.encode_data_block_image(entries))
        img[sst.CRC_OFFSET:sst.CRC_OFFSET + 4] = rng.bytes(4)  # whatever the field holds
        zeroed = bytes(img[:17]) + bytes(4) + bytes(img[21:])
        assert oracle.sst_stamp(bytes(img)) == zlib.crc32(zeroed)


def test_sst_image_layout():
    """get_data_block's image (sstable_writer.cpp:137-168): varint(20) | header | varint(n) | body,
    allocated as 8 + 20 + 8 + n bytes; header fields per sstable_format.hpp:91-99."""
    import struct
    import tinykvpp_amd.sst as sst
    entries = [(b"key1", b"value1"), (b"k2", b"v")]
    img = sst.encode_data_block_image(entries)
    n = (8 + 4 + 6) + (8 + 2 + 1)
    assert len(img) == 8 + 20 + 8 + n
    assert img[0] == 20
    count, usize, csize, comp, crc = struct.unpack_from("<IIIB3xI", img, 1)
    assert (count, usize, csize, comp, crc) == (2, n, n, 0, 0)
    assert img[21] == n and img[22:22 + 5] == b"\x04key1"
    assert sst.CRC_OFFSET == 1 + 16


def test_fast_synthetic_path_matches_sarwate(oracle):
    """oracle_crc_synthetic_s8 (used to checksum whole shards on CPU) == the Sarwate restatement on
    the golden first blocks and on lengths that exercise its byte tail."""
    g = golden("synthetic.json")
    fn = oracle.lib.oracle_crc_synthetic_s8
    fn.argtypes = [ctypes.c_uint64] * 4 + [ctypes.c_void_p]
    for cfg in ("cfg2", "cfg3"):
        out = np.zeros(64, np.uint32)
        fn(1, 0, 64, g[cfg]["len"], out.ctypes.data)
        assert [int(x) for x in out] == g[cfg]["first"]
    for n in (0, 1, 3, 7, 8, 9, 255, 4097):
        out = np.zeros(8, np.uint32)
        fn(1, 100, 8, n, out.ctypes.data)
        assert np.array_equal(out, oracle.synthetic(1, 100, 8, n))


def test_shard_fixtures_are_consistent():
    """Per-rank shard aggregates (make_golden.py --shards): rank 0's shard of cfg2/cfg3/cfg4 is the
    whole single-GPU config, and the eight cfg5 shards recombine into the survey's 4 M x 64 KiB
    aggregate (XOR 5a7eaa3b, SUM32 9d26ebfd)."""
    g = golden("synthetic.json")
    sh = g["shards"]
    for cfg in ("cfg2", "cfg3", "cfg4"):
        assert len(sh[cfg]) == 8
        assert (sh[cfg][0]["xor"], sh[cfg][0]["sum32"]) == (g[cfg]["xor"], g[cfg]["sum32"])
        assert [s["first_block"] for s in sh[cfg]] == [r * g[cfg]["nblocks"] for r in range(8)]
    x = s = 0
    for r, shard in enumerate(sh["cfg5"]):
        assert shard["first_block"] == r * (1 << 19) and shard["nblocks"] == 1 << 19
        x ^= shard["xor"]
        s = (s + shard["sum32"]) & 0xFFFFFFFF
    assert (x, s) == (0x5A7EAA3B, 0x9D26EBFD) == (g["cfg5"]["xor"], g["cfg5"]["sum32"])


def test_reference_wal_loops(ref_lib):
    """oracle/_ref's restatement of the reference's recovery loop (wal_entry::decode until the image
    ends, wal.cpp:63-130) and encode stamp (wal.cpp:54-58) over the reference's own crc32.cpp: the
    CPU path tools/bench_formats.py times beside the GPU rows. Pinned by the golden records
    (tests/golden/wal.json, written from the compiled reference)."""
    import ctypes
    recs = [bytes.fromhex(r["hex"]) for r in golden("wal.json")["records"]]
    img = bytearray(b"".join(recs))
    good, stop = ctypes.c_uint64(), ctypes.c_uint64()
    ref_lib.ref_wal_verify.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
    ref_lib.ref_wal_stamp.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]

    def verify(b):
        rc = ref_lib.ref_wal_verify(bytes(b), len(b), ctypes.byref(good), ctypes.byref(stop))
        return rc, good.value, stop.value

    assert verify(img) == (0, len(recs), len(img))
    starts = np.cumsum([0] + [len(r) for r in recs])
    bad = bytearray(img)
    bad[int(starts[3]) + 20] ^= 0x40  # a CRC-covered byte of record 3 (its key_len): CRC mismatch there
    assert verify(bad) == (4, 3, int(starts[3]))
    assert verify(img[:-1]) == (4, len(recs) - 1, int(starts[-2]))  # torn tail
    zeroed = bytearray(img)
    for s in starts[:-1]:
        zeroed[int(s) + 4:int(s) + 8] = b"\0\0\0\0"
    offs = np.array(starts[:-1], np.uint64)
    sizes = np.array([len(r) for r in recs], np.uint32)
    buf = ctypes.create_string_buffer(bytes(zeroed), len(zeroed))
    ref_lib.ref_wal_stamp(buf, offs.ctypes.data, sizes.ctypes.data, len(recs))
    assert buf.raw[:len(img)] == bytes(img)


def _wal_oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import wal_images
    return wal_images, wal_images.load()


def _py_decode(img):
    """wal.cpp:63-130 applied record after record, in Python (the tests' sequential decode)."""
    import zlib
    u32 = lambda p: int.from_bytes(bytes(img[p:p + 4]), "little")  # noqa: E731
    p, n, size = 0, 0, len(img)
    while p < size:
        if size - p < 26 or u32(p) + 8 > size - p:
            return "corrupted", n, p
        rl = u32(p)
        if zlib.crc32(bytes(img[p + 8:p + 8 + rl])) != u32(p + 4) or 26 + u32(p + 18) + u32(p + 22) > 8 + rl:
            return "corrupted", n, p
        p += 8 + rl
        n += 1
    return "ok", n, p


def test_oracle_wal_decode_golden():
    """oracle_wal_decode / oracle_wal_stamp (the checker bench.py's bit_exact_paths and smoke() use)
    on the reference's golden records (tests/golden/wal.json, written from the compiled reference):
    clean, a flipped CRC-covered byte, a torn tail, a key_len past the record, restamping."""
    wi, wo = _wal_oracle()
    recs = [bytes.fromhex(r["hex"]) for r in golden("wal.json")["records"]]
    img = np.frombuffer(b"".join(recs), np.uint8).copy()
    starts = np.cumsum([0] + [len(r) for r in recs]).astype(np.uint64)
    assert wi.decode(wo, img) == ("ok", len(recs), img.size)
    bad = img.copy()
    bad[int(starts[3]) + 20] ^= 0x40
    assert wi.decode(wo, bad) == ("corrupted", 3, int(starts[3]))
    assert wi.decode(wo, img, img.size - 1) == ("corrupted", len(recs) - 1, int(starts[-2]))
    assert wi.decode(wo, img, 0) == ("ok", 0, 0)
    un = img.copy()
    for s in starts[:-1]:
        un[int(s) + 4:int(s) + 8] = 0
    st0 = starts[:-1].copy()
    wo.oracle_wal_stamp(un.ctypes.data, st0.ctypes.data, len(recs))
    assert np.array_equal(un, img)
    # key_len + value_len past the record (restamped so only the bounds check fails, wal.cpp:115-119)
    kv = img.copy()
    kv[int(starts[2]) + 18:int(starts[2]) + 22] = np.frombuffer((10 ** 6).to_bytes(4, "little"), np.uint8)
    st2 = starts[2:3].copy()
    wo.oracle_wal_stamp(kv.ctypes.data, st2.ctypes.data, 1)
    assert wi.decode(wo, kv) == ("corrupted", 2, int(starts[2])) == _py_decode(kv)


@pytest.mark.parametrize("shape", ["small", "zipf", "values_of_records"])
def test_oracle_wal_images(shape):
    """The synthetic images (oracle/wal_images.py) decode clean; one flipped payload byte, a lying
    record_len and a truncation stop where the Python decode (zlib CRC) stops."""
    wi, wo = _wal_oracle()
    img, offs, size = wi.image(wo, shape, 3000, seed=7)
    assert wi.decode(wo, img) == ("ok", 3000, img.size) == _py_decode(img)
    for victim in (0, 1500, 2999):
        b = img.copy()
        b[int(offs[victim] + size[victim] - 1)] ^= 1
        assert wi.decode(wo, b) == ("corrupted", victim, int(offs[victim])) == _py_decode(b)
        b = img.copy()
        b[int(offs[victim]):int(offs[victim]) + 4] = np.frombuffer((int(size[victim]) - 8 + 3).to_bytes(4, "little"),
                                                                   np.uint8)
        assert wi.decode(wo, b) == _py_decode(b)
    assert wi.decode(wo, img, img.size - 3) == _py_decode(img[:-3])


def test_oracle_wal_decode_matches_reference(ref_lib):
    """oracle_wal_decode against oracle/_ref's ref_wal_verify (the reference's own crc32.cpp) on the
    synthetic images, clean and corrupted."""
    wi, wo = _wal_oracle()
    ref_lib.ref_wal_verify.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
    for shape in ("small", "zipf", "values_of_records"):
        img, offs, size = wi.image(wo, shape, 20000, seed=11)
        for flip in (None, int(offs[12345]) + 30):
            b = img.copy()
            if flip is not None:
                b[flip] ^= 0x20
            good, stop = ctypes.c_uint64(), ctypes.c_uint64()
            rc = ref_lib.ref_wal_verify(b.ctypes.data, b.size, ctypes.byref(good), ctypes.byref(stop))
            assert wi.decode(wo, b) == ("corrupted" if rc else "ok", good.value, stop.value)
