"""Record-list check of a WAL image in HBM (tkv_wal_check_records_device; tinykvpp_amd.wal.check_records_device).

Records whose start offsets are known are checked as wal_entry::decode checks one record
(/root/reference/src/engine/wal.cpp:63-127): at least 26 bytes left, record_len + 8 within the
image, CRC-32 of the payload equal to the stored CRC, key and value inside the payload. Every case is
compared record by record with a restatement of those checks here, the CRC from the test oracle
(crc32.cpp:9-16 restated), so parity is against the reference's decode, not the library's own
paths. Images are the reference's WAL layout (wal.cpp:19-61) stamped by tkv_wal_stamp and checked
against the golden records of tests/golden/wal.json.
"""
import numpy as np
import pytest
import torch

import tinykvpp_amd as tk
from conftest import golden
from test_gpu_wal_device import make_wal

pytestmark = pytest.mark.gpu


def u32at(img, p):
    return int.from_bytes(img[p:p + 4].tobytes(), "little")


def expected(oracle, img, size, offs):
    """Per record: (computed CRC or 0 when its length check fails, ok)."""
    offs = np.asarray(offs, np.int64)
    n = offs.size
    crc = np.zeros(n, np.uint32)
    ok = np.zeros(n, bool)
    left = np.where(offs < size, size - offs, 0)
    hdr = left >= 26
    idx = np.flatnonzero(hdr)
    rlen = np.zeros(n, np.int64)
    if idx.size:
        o = offs[idx]
        b = img[(o[:, None] + np.arange(26)).astype(np.int64)]
        rl = b[:, 0:4].copy().view("<u4").reshape(-1).astype(np.int64)
        rlen[idx] = rl
    len_ok = hdr & (rlen + 8 <= left)
    li = np.flatnonzero(len_ok)
    if li.size:
        o = offs[li]
        crc[li] = oracle.batch(img, (o + 8).astype(np.uint64), rlen[li].astype(np.uint32))
        b = img[(o[:, None] + np.arange(26)).astype(np.int64)]
        stored = b[:, 4:8].copy().view("<u4").reshape(-1)
        klen = b[:, 18:22].copy().view("<u4").reshape(-1).astype(np.int64)
        vlen = b[:, 22:26].copy().view("<u4").reshape(-1).astype(np.int64)
        ok[li] = (crc[li] == stored) & (18 + klen + vlen <= rlen[li])
    return crc, ok


def run(img, offs, max_payload, shift=0, gpu="cuda:0"):
    d = torch.zeros(img.size + shift, dtype=torch.uint8, device=gpu)
    if img.size:
        d[shift:] = torch.from_numpy(img).to(gpu)
    o = torch.from_numpy(np.asarray(offs, np.int64).astype(np.uint32).view(np.int32)).to(gpu)
    fb, crc = tk.wal.check_records_device(d[shift:], o, max_payload=max_payload)
    torch.cuda.synchronize()
    return int(fb.item()), crc.cpu().numpy().view(np.uint32)


def check(oracle, img, offs, max_payload, shift=0):
    first, crc = run(img, offs, max_payload, shift)
    want_crc, ok = expected(oracle, img, img.size, offs)
    bad = np.flatnonzero(~ok)
    assert first == (int(bad[0]) if bad.size else len(offs)), (first, bad[:5])
    diff = np.flatnonzero(crc != want_crc)
    assert diff.size == 0, f"{diff.size} CRCs differ, first {diff[:5]}"
    return first


def make_wal_small(rng, n):
    """Records of the reference's per-put shape: 26 + |k| + |v| bytes, |k| 4-23, |v| 0-39 (payloads
    of 22-80 bytes, tools/ab_wal.py's 1 GiB image), stamped."""
    import ctypes
    klen = rng.integers(4, 24, n).astype(np.uint64)
    vlen = rng.integers(0, 40, n).astype(np.uint64)
    size = 26 + klen + vlen
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(size[:-1])
    img = rng.integers(0, 256, int(size.sum()), dtype=np.uint8)
    hdr = np.zeros((n, 26), np.uint8)
    hdr[:, 0:4] = (size - 8).astype("<u4").view(np.uint8).reshape(-1, 4)
    hdr[:, 18:22] = klen.astype("<u4").view(np.uint8).reshape(-1, 4)
    hdr[:, 22:26] = vlen.astype("<u4").view(np.uint8).reshape(-1, 4)
    img[offs.astype(np.int64)[:, None] + np.arange(26)] = hdr
    s32 = size.astype(np.uint32)
    tk.check(tk.load_library().tkv_wal_stamp(ctypes.c_void_p(img.ctypes.data), ctypes.c_void_p(offs.ctypes.data),
                                             ctypes.c_void_p(s32.ctypes.data), n))
    return img, offs, size


def test_golden_records(gpu, oracle):
    recs = [bytes.fromhex(r["hex"]) for r in golden("wal.json")["records"]]
    img = np.frombuffer(b"".join(recs), np.uint8).copy()
    offs = np.concatenate([[0], np.cumsum([len(r) for r in recs])[:-1]])
    for mp in (64, 100, 4096):
        first, crc = run(img, offs, mp)
        assert first == len(recs)
        assert crc.tolist() == [r["crc"] for r in golden("wal.json")["records"]]


@pytest.mark.parametrize("max_payload", [36, 50, 64, 80, 100, 1024])
@pytest.mark.parametrize("shift", [0, 3, 8, 13])
def test_small_records_every_alignment(gpu, oracle, max_payload, shift):
    rng = np.random.default_rng(shift * 7 + max_payload)
    img, offs, _ = make_wal_small(rng, 60_000)
    assert check(oracle, img, offs, max_payload, shift) == offs.size


@pytest.mark.parametrize("max_payload", [64, 2000])
def test_zipf_records_long_payloads(gpu, oracle, max_payload):
    """Values up to 16 KB: payloads far past the window continue 64 bytes at a time, exact."""
    rng = np.random.default_rng(max_payload)
    img, offs, _ = make_wal(rng, 20_000)
    assert check(oracle, img, offs, max_payload, 5) == offs.size


def test_every_payload_length(gpu, oracle):
    """Payloads of every length 18..300 (records 26..308 bytes) at every start alignment."""
    import ctypes
    rng = np.random.default_rng(3)
    sizes = np.tile(np.arange(26, 309, dtype=np.uint64), 17)
    rng.shuffle(sizes)
    n = sizes.size
    klen = np.minimum(sizes - 26, rng.integers(0, 30, n).astype(np.uint64))
    vlen = sizes - 26 - klen
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(sizes[:-1])
    img = rng.integers(0, 256, int(sizes.sum()), dtype=np.uint8)
    hdr = np.zeros((n, 26), np.uint8)
    hdr[:, 0:4] = (sizes - 8).astype("<u4").view(np.uint8).reshape(-1, 4)
    hdr[:, 18:22] = klen.astype("<u4").view(np.uint8).reshape(-1, 4)
    hdr[:, 22:26] = vlen.astype("<u4").view(np.uint8).reshape(-1, 4)
    img[offs.astype(np.int64)[:, None] + np.arange(26)] = hdr
    s32 = sizes.astype(np.uint32)
    tk.check(tk.load_library().tkv_wal_stamp(ctypes.c_void_p(img.ctypes.data), ctypes.c_void_p(offs.ctypes.data),
                                             ctypes.c_void_p(s32.ctypes.data), n))
    for mp in (36, 64, 80, 100, 300):
        assert check(oracle, img, offs, mp, 1) == n


@pytest.mark.parametrize("kind", ["payload_bit", "stored_crc", "kv_overrun", "record_len_lies", "offset_past_end",
                                  "tail_too_short", "first_record", "several"])
def test_corruptions(gpu, oracle, kind):
    """Each check of wal_entry::decode fails on its own (wal.cpp:68, :80, :89-96, :118-121), and the
    first failing record is reported; the other records' CRCs stay exact."""
    rng = np.random.default_rng(sum(map(ord, kind)))
    img, offs, size = make_wal_small(rng, 30_000)
    offs = offs.astype(np.int64)
    size = size.astype(np.int64)
    i = int(rng.integers(100, offs.size - 100))
    want = i
    if kind == "payload_bit":
        img[offs[i] + 8 + int(rng.integers(0, size[i] - 8))] ^= 1 << int(rng.integers(0, 8))
    elif kind == "stored_crc":
        img[offs[i] + 5] ^= 0x40
    elif kind == "kv_overrun":  # key length past the payload, CRC restamped: only the bounds check fails
        img[offs[i] + 18:offs[i] + 22] = np.frombuffer((int(size[i]) + 5).to_bytes(4, "little"), np.uint8)
        payload = img[offs[i] + 8:offs[i] + size[i]].tobytes()
        img[offs[i] + 4:offs[i] + 8] = np.frombuffer(oracle.crc(payload).to_bytes(4, "little"), np.uint8)
    elif kind == "record_len_lies":  # longer than what is left of the image
        img[offs[i]:offs[i] + 4] = np.frombuffer((img.size).to_bytes(4, "little"), np.uint8)
    elif kind == "offset_past_end":
        offs = offs.copy()
        offs[i] = img.size + 3
    elif kind == "tail_too_short":  # the last record starts fewer than 26 bytes before the end
        offs = np.append(offs, img.size - 20)
        want = offs.size - 1
    elif kind == "first_record":
        img[offs[0] + 30] ^= 0x80
        want = 0
    else:  # several: the lowest index wins
        for j in (i + 50, i, i + 7):
            img[offs[j] + 9] ^= 0x01
    assert check(oracle, img, offs, 64, 0) == want
    assert check(oracle, img, offs, 100, 7) == want


def test_empty_and_tiny(gpu, oracle):
    first, _ = run(np.zeros(0, np.uint8), np.zeros(0, np.int64), 64)
    assert first == 0
    img, offs, _ = make_wal_small(np.random.default_rng(9), 1)
    assert check(oracle, img, offs, 64) == 1
    assert check(oracle, img[:-1].copy(), offs, 64) == 0  # record_len overruns the truncated image


def make_wal_sized(rng, sizes):
    """Stamped records of the given total sizes (26 + |k| + |v| each)."""
    import ctypes
    sizes = np.asarray(sizes, np.uint64)
    n = sizes.size
    klen = np.minimum(sizes - 26, rng.integers(0, 12, n).astype(np.uint64))
    vlen = sizes - 26 - klen
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(sizes[:-1])
    img = rng.integers(0, 256, int(sizes.sum()), dtype=np.uint8)
    hdr = np.zeros((n, 26), np.uint8)
    hdr[:, 0:4] = (sizes - 8).astype("<u4").view(np.uint8).reshape(-1, 4)
    hdr[:, 18:22] = klen.astype("<u4").view(np.uint8).reshape(-1, 4)
    hdr[:, 22:26] = vlen.astype("<u4").view(np.uint8).reshape(-1, 4)
    img[offs.astype(np.int64)[:, None] + np.arange(26)] = hdr
    s32 = sizes.astype(np.uint32)
    tk.check(tk.load_library().tkv_wal_stamp(ctypes.c_void_p(img.ctypes.data), ctypes.c_void_p(offs.ctypes.data),
                                             ctypes.c_void_p(s32.ctypes.data), n))
    return img, offs


@pytest.mark.parametrize("layout", ["uniform_44", "mixed_spans", "permuted", "to_the_end"])
@pytest.mark.parametrize("shift", [0, 3, 8, 13])
def test_lds_staged_windows(gpu, oracle, layout, shift):
    """Windows of 4-5 granules with payloads of at least 32 bytes are staged through LDS a step at a
    time: 44-byte records (every step staged); steps holding a long record next to
    staged ones (its span over 3 KiB: that step loads granules); offsets out of order (spans over 3 KiB
    everywhere); the last records ending on the image's last byte. Payload flips in staged steps must
    report the first bad record."""
    rng = np.random.default_rng(len(layout) * 31 + shift)
    n = 20_000
    sizes = np.full(n, 44, np.uint64)
    if layout == "mixed_spans":
        sizes[rng.integers(0, n, 60)] = rng.integers(1500, 5000, 60).astype(np.uint64)
        sizes[rng.integers(0, n, 2000)] = rng.integers(40, 81, 2000).astype(np.uint64)
    img, offs = make_wal_sized(rng, sizes)
    if layout == "permuted":
        offs = offs[rng.permutation(n)]
    for mp in (36, 54):
        assert check(oracle, img, offs, mp, shift) == n
    if layout != "permuted":
        o = offs.astype(np.int64)
        for i in sorted(rng.integers(70, n - 70, 3), reverse=True):  # latest first: each becomes the first bad
            img[o[i] + 8 + int(rng.integers(0, 36))] ^= 0x10
            assert check(oracle, img, offs, 36, shift) == i


@pytest.mark.parametrize("max_payload", [36, 64])
def test_null_crc_output(gpu, oracle, max_payload):
    """d_crc = NULL through the C ABI: only the first bad record is computed, on the
    LDS-staged path (36-byte payloads, 4-granule windows) and the granule path; clean and with a CRC
    flip, first_bad must equal the restated decode's."""
    import ctypes
    rng = np.random.default_rng(77 + max_payload)
    n = 20000
    klen = rng.integers(0, 6, n).astype(np.uint64)
    vlen = (max_payload - 18 - klen).astype(np.uint64)
    size = 26 + klen + vlen
    offs = np.concatenate([[0], np.cumsum(size[:-1])]).astype(np.uint64)
    img = rng.integers(0, 256, int(size.sum()), dtype=np.uint8)
    hdr = np.zeros((n, 26), np.uint8)
    hdr[:, 0:4] = (size - 8).astype("<u4").view(np.uint8).reshape(-1, 4)
    hdr[:, 18:22] = klen.astype("<u4").view(np.uint8).reshape(-1, 4)
    hdr[:, 22:26] = vlen.astype("<u4").view(np.uint8).reshape(-1, 4)
    img[offs.astype(np.int64)[:, None] + np.arange(26)] = hdr
    size32 = size.astype(np.uint32)
    lib = tk.load_library()
    tk.check(lib.tkv_wal_stamp(ctypes.c_void_p(img.ctypes.data), ctypes.c_void_p(offs.ctypes.data),
                               ctypes.c_void_p(size32.ctypes.data), n))
    for flip in (None, 12345):
        if flip is not None:
            img[int(offs[flip]) + int(size[flip]) - 1] ^= 0x10
        _, ok = expected(oracle, img, img.size, offs)
        bad = np.flatnonzero(~ok)
        want = int(bad[0]) if bad.size else n
        d = torch.from_numpy(img).cuda()
        o = torch.from_numpy(offs.astype(np.uint32).view(np.int32)).cuda()
        fb = torch.empty(1, dtype=torch.int64, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        tk.check(lib.tkv_wal_check_records_device(ctypes.c_void_p(d.data_ptr()), img.size,
                                                  ctypes.c_void_p(o.data_ptr()), n, max_payload, None,
                                                  ctypes.c_void_p(fb.data_ptr()), ctypes.c_void_p(st)))
        torch.cuda.synchronize()
        assert int(fb.item()) == want, (flip, int(fb.item()), want)
