"""GPU parity for the §8f rows beyond the WAL: CRC-32C on the same engine and SSTable data-block
stamping. CRC-32C is checked against the oracle restatement pinned by RFC 3720 §B.4; the SSTable
stamp against the oracle's literal zero-field CRC (the format is this library's: parity unpinned
by the reference, whose crc32_ fields stay 0, sstable_writer.cpp:138-144)."""
import numpy as np
import pytest

import tinykvpp_amd as tk
import tinykvpp_amd.sst as sst
from test_oracle import RFC3720_B4

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def u32(t):
    return t.cpu().numpy().view(np.uint32)


# ---- CRC-32C ----------------------------------------------------------------------------------------

@pytest.mark.parametrize("data,want", RFC3720_B4)
def test_crc32c_published_vectors(gpu, data, want):
    assert tk.crc32c().update(data).finalize() == want


def test_crc32c_incremental_and_device(gpu, oracle):
    rng = np.random.default_rng(11)
    data = rng.bytes(300_000)
    c = tk.crc32c()
    for a, b in ((0, 7), (7, 70_001), (70_001, 300_000)):
        c = c.update(data[a:b])
    assert c.finalize() == oracle.crc_c(data)
    t = torch.from_numpy(np.frombuffer(data, np.uint8).copy()).to(gpu)
    assert tk.crc32c().update(t).finalize() == oracle.crc_c(data)


@pytest.mark.parametrize("blen,n", [(4096, 300_000), (65536, 4096), (1000, 5000), (4100, 777)])
def test_crc32c_uniform(gpu, oracle, blen, n):
    """(4096, 300 000) and (65536, 4096) take the packed kernel; the others the generic rows."""
    rng = np.random.default_rng(blen)
    host = rng.integers(0, 256, blen * n, dtype=np.uint8)
    got = u32(tk.crc32_batch_uniform(torch.from_numpy(host).to(gpu), blen, n, algo="crc32c"))
    idx = rng.integers(0, n, 64)
    for i in idx:
        assert int(got[i]) == oracle.crc_c(host[i * blen:(i + 1) * blen].tobytes())


def test_crc32c_irregular_and_host(gpu, oracle):
    rng = np.random.default_rng(7)
    lens = rng.integers(0, 20_000, 3000).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.int64))]) + rng.integers(0, 3, lens.size).cumsum()
    host = rng.integers(0, 256, int(offs[-1] + lens[-1] + 8), dtype=np.uint8)
    want = np.array([oracle.crc_c(host[o:o + l].tobytes()) for o, l in zip(offs, lens)], np.uint32)
    d = torch.from_numpy(host).to(gpu)
    got = u32(tk.crc32_batch(d, torch.from_numpy(offs.astype(np.int64)).to(gpu),
                             torch.from_numpy(lens.astype(np.int32)).to(gpu), algo="crc32c"))
    assert np.array_equal(got, want)
    assert np.array_equal(tk.crc32_batch_host(host, offs.astype(np.uint64), lens, algo="crc32c"), want)
    assert np.array_equal(tk.crc32_batch_host(host, offs.astype(np.uint64), lens, algo="crc32c", devices=[0, 0]), want)
    # the two families really differ
    assert not np.array_equal(tk.crc32_batch_host(host, offs.astype(np.uint64), lens), want)


# ---- SSTable data-block stamping ----------------------------------------------------------------------

def make_file(rng, nblocks):
    """An SSTable-like file image: data-block images back to back (sstable_writer.cpp:131-169)."""
    imgs = []
    for _ in range(nblocks):
        entries = [(rng.bytes(int(rng.integers(8, 40))), rng.bytes(int(rng.integers(0, 300))))
                   for _ in range(int(rng.integers(1, 30)))]
        imgs.append(sst.encode_data_block_image(entries))
    sizes = np.array([len(i) for i in imgs], np.uint64)
    offs = np.concatenate([[0], np.cumsum(sizes[:-1])]).astype(np.uint64)
    return np.frombuffer(b"".join(imgs), np.uint8).copy(), offs, sizes


def test_sst_stamp_matches_oracle_and_verifies(gpu, oracle):
    rng = np.random.default_rng(21)
    f, offs, sizes = make_file(rng, 500)
    sst.stamp_blocks(f, offs, sizes)
    for o, s in zip(offs[::7], sizes[::7]):
        img = f[int(o):int(o + s)].tobytes()
        assert int.from_bytes(img[17:21], "little") == oracle.sst_stamp(img)
    assert sst.verify_blocks(f, offs, sizes) == ("ok", 0, 500)


@pytest.mark.parametrize("where", ["varint", "header", "crc_field", "body", "padding"])
def test_sst_corruption_detected(gpu, where):
    rng = np.random.default_rng(22)
    f, offs, sizes = make_file(rng, 64)
    sst.stamp_blocks(f, offs, sizes)
    victim = 41
    o, s = int(offs[victim]), int(sizes[victim])
    pos = {"varint": 0, "header": 5, "crc_field": 19, "body": 30, "padding": s - 1}[where]
    f[o + pos] ^= 0x10
    assert sst.verify_blocks(f, offs, sizes) == ("corrupted", 1, victim)


def test_sst_device_stamp_equals_host_stamp(gpu):
    rng = np.random.default_rng(23)
    f, offs, sizes = make_file(rng, 2000)
    host = f.copy()
    sst.stamp_blocks(host, offs, sizes)
    f[offs.astype(np.int64)[:, None] + np.arange(17, 21)] = rng.integers(0, 256, (offs.size, 4), dtype=np.uint8)
    d = torch.from_numpy(f).to(gpu)
    o = torch.from_numpy(offs.astype(np.int64)).to(gpu)
    sz = torch.from_numpy(sizes.astype(np.int32)).to(gpu)
    vals = u32(sst.block_crcs_device(d, o, sz))          # whatever the fields hold
    want = host[offs.astype(np.int64)[:, None] + np.arange(17, 21)].copy().view("<u4").ravel()
    assert np.array_equal(vals, want)
    sst.block_crcs_device(d, o, sz, store=True)           # stamp on the device
    assert np.array_equal(d.cpu().numpy(), host)
    assert sst.verify_blocks(d.cpu().numpy(), offs, sizes)[0] == "ok"


def test_sst_device_checks_its_tensors(gpu):
    """block_crcs_device checks shapes, dtypes and devices before any launch: a short `out`, a
    length mismatch or a non-uint8 file would otherwise become an out-of-bounds device access."""
    rng = np.random.default_rng(24)
    f, offs, sizes = make_file(rng, 16)
    d = torch.from_numpy(f).to(gpu)
    o = torch.from_numpy(offs.astype(np.int64)).to(gpu)
    sz = torch.from_numpy(sizes.astype(np.int32)).to(gpu)
    for kw in ({"out": torch.empty(15, dtype=torch.int32, device=gpu)},
               {"out": torch.empty(16, dtype=torch.int64, device=gpu)}):
        with pytest.raises(ValueError):
            sst.block_crcs_device(d, o, sz, **kw)
    with pytest.raises(ValueError):
        sst.block_crcs_device(d, o, sz[:15])
    with pytest.raises(ValueError):
        sst.block_crcs_device(d.view(torch.int8), o, sz)
    with pytest.raises(ValueError):
        sst.block_crcs_device(d, o.to(torch.int32), sz)
    assert u32(sst.block_crcs_device(d, o, sz)).size == 16


def test_sst_rejects_short_images(gpu):
    f = np.zeros(100, np.uint8)
    with pytest.raises(tk.TkvError):
        sst.stamp_blocks(f, [0], [21])


def test_sst_and_wal_on_pinned_buffers(gpu, oracle):
    """SSTable stamp/verify and WAL stamp/verify over pinned images (read in place by the kernels):
    identical to the pageable path, corruption still detected."""
    import ctypes
    rng = np.random.default_rng(31)
    nblk, size = 300, 4096
    img = rng.integers(0, 256, nblk * size, dtype=np.uint8)
    offs = np.arange(nblk, dtype=np.uint64) * size
    sizes = np.full(nblk, size, np.uint64)
    img[offs.astype(np.int64)] = 20
    ref = img.copy()
    sst.stamp_blocks(ref, offs, sizes)
    keep = torch.from_numpy(img).pin_memory()
    pin = keep.numpy()
    sst.stamp_blocks(pin, offs, sizes)
    assert np.array_equal(pin, ref)
    assert sst.verify_blocks(pin, offs, sizes)[0] == "ok"
    pin[5 * size + 100] ^= 1
    assert sst.verify_blocks(pin, offs, sizes)[:3] == ("corrupted", 1, 5)
    pin[5 * size + 100] ^= 1
    sst.stamp_blocks(pin, offs, sizes)  # restamping a stamped image gives the same stamps
    assert np.array_equal(pin, ref)
    # WAL group-commit stamp and recovery verify over a pinned append buffer
    recs = [tk.wal.encode_unstamped(i % 2, i, rng.bytes(int(rng.integers(0, 40))), rng.bytes(int(rng.integers(0, 900))),
                                    i % 2) for i in range(2000)]
    want = b"".join(tk.wal.stamp(recs))
    sz = np.array([len(r) for r in recs], np.uint32)
    of = np.zeros(len(recs), np.uint64)
    of[1:] = np.cumsum(sz[:-1], dtype=np.uint64)
    wk = torch.from_numpy(np.frombuffer(b"".join(recs), np.uint8).copy()).pin_memory()
    wp = wk.numpy()
    lib = tk.load_library()
    tk.check(lib.tkv_wal_stamp(ctypes.c_void_p(wp.ctypes.data), ctypes.c_void_p(of.ctypes.data),
                               ctypes.c_void_p(sz.ctypes.data), len(recs)))
    assert wp.tobytes() == want
    good, stop = ctypes.c_uint64(0), ctypes.c_uint64(0)
    assert lib.tkv_wal_verify(ctypes.c_void_p(wp.ctypes.data), wp.size, ctypes.byref(good), ctypes.byref(stop)) == 0
    assert (good.value, stop.value) == (len(recs), wp.size)
    wp[int(of[700]) + 30] ^= 0x40  # payload byte of record 700 (every record is >= 26 bytes... key/value)
    rc = lib.tkv_wal_verify(ctypes.c_void_p(wp.ctypes.data), wp.size, ctypes.byref(good), ctypes.byref(stop))
    assert rc != 0 and good.value <= 700 and stop.value <= int(of[700])


# ---- SSTable index image + footer (format: include/tkv_crc32.h; parity unpinned) ------------------

def make_index(rng, offs, sizes):
    """Index entries as sstable_writer::record_data_block records them (smallest key, offset, size)."""
    return sst.encode_index_image([(rng.bytes(int(rng.integers(1, 64))), int(o), int(s))
                                   for o, s in zip(offs, sizes)])


@pytest.mark.parametrize("nblocks", [0, 1, 37, 3000])
def test_sst_footer_stamp_matches_oracle(gpu, oracle, nblocks):
    rng = np.random.default_rng(100 + nblocks)
    _, offs, sizes = make_file(rng, max(nblocks, 1))
    index = make_index(rng, offs[:nblocks], sizes[:nblocks]) if nblocks else b""
    index_offset = int(offs[-1] + sizes[-1])
    footer = sst.stamp_footer(index, sst.encode_footer(index_offset, len(index)))
    want = oracle.crc(index + footer[:16])
    assert int.from_bytes(footer[16:20], "little") == want
    assert footer[:16] == sst.encode_footer(index_offset, len(index))[:16]
    assert sst.verify_footer(index, footer) == "ok"


def test_sst_footer_detects_index_and_field_corruption(gpu):
    rng = np.random.default_rng(5)
    _, offs, sizes = make_file(rng, 200)
    index = bytearray(make_index(rng, offs, sizes))
    footer = bytearray(sst.stamp_footer(bytes(index), sst.encode_footer(123456, len(index), 7, 8)))
    for pos in (0, 8, len(index) // 2, len(index) - 1):          # count, first key, an offset, last size
        bad = bytearray(index)
        bad[pos] ^= 0x10
        assert sst.verify_footer(bytes(bad), bytes(footer)) == "corrupted"
    for pos in (0, 5, 9, 13, 17):                                # each footer field, crc32_ itself
        bad = bytearray(footer)
        bad[pos] ^= 1
        assert sst.verify_footer(bytes(index), bytes(bad)) == "corrupted"
    assert sst.verify_footer(bytes(index[:-1]), bytes(footer)) == "corrupted"   # truncated index
    with pytest.raises(ValueError):
        sst.stamp_footer(bytes(index), bytes(footer[:16]))


def test_sst_whole_file_roundtrip(gpu):
    """A whole SSTable image: data blocks, index, footer (sstable_writer flush order). Every block
    and the index/footer stamped on the GPU, then verified from the file bytes alone."""
    rng = np.random.default_rng(8)
    f, offs, sizes = make_file(rng, 400)
    sst.stamp_blocks(f, offs, sizes)
    index = make_index(rng, offs, sizes)
    footer = sst.stamp_footer(index, sst.encode_footer(f.size, len(index)))
    image = f.tobytes() + index + footer
    # reader side: footer first (sstable_reader.cpp:19-38), then the index it points to, then blocks
    foot = image[-sst.FOOTER_SIZE:]
    io, isz = int.from_bytes(foot[0:4], "little"), int.from_bytes(foot[4:8], "little")
    assert sst.verify_footer(image[io:io + isz], foot) == "ok"
    assert sst.verify_blocks(np.frombuffer(image, np.uint8), offs, sizes) == ("ok", 0, 400)
