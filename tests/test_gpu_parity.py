"""GPU parity: the HIP path (through the C ABI) against the oracle and the reference's golden vectors.

Bit-exact on every block. Small sizes are compared block by block with the oracle; the BASELINE
configs at full size are compared through their golden aggregates (XOR and SUM32 of all block
CRCs), plus properties (incremental == single, corruption always detected).
"""
import struct

import numpy as np
import pytest

import tinykvpp_amd as tk
from conftest import golden

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def dev_bytes(b, device):
    a = np.frombuffer(bytes(b), np.uint8)
    return torch.from_numpy(a.copy()).to(device) if a.size else torch.empty(0, dtype=torch.uint8, device=device)


# ---- crc32_test.cpp:81-124 through the reference-shaped class ------------------------------------

def test_known_answers(gpu):
    k = golden("kat.json")
    assert tk.crc32().finalize() == 0  # EmptyInput
    for s in k["strings"]:
        assert tk.crc32().update(s["text"].encode()).finalize() == s["crc"]
    assert tk.crc32().update(b"123456789").finalize() == 0xCBF43926
    assert tk.crc32().update(b"The quick brown fox jumps over the lazy dog").finalize() == 0x414FA339


def test_incremental_equals_single(gpu):
    data = b"Hello, World!"
    single = tk.crc32().update(data).finalize()
    c = tk.crc32()
    c.update(data[:5]).update(data[5:7]).update(data[7:])
    assert c.finalize() == single == golden("kat.json")["incremental"]["crc"]
    c.reset()
    assert c.finalize() == 0


def test_update_device_tensor(gpu, oracle):
    rng = np.random.default_rng(1)
    for n in (0, 1, 3, 4, 5, 64, 4095, 4096, 4097, 100003, 3 << 20):
        d = rng.integers(0, 256, n, dtype=np.uint8)
        t = torch.from_numpy(d).to(gpu)
        assert tk.crc32().update(t).finalize() == oracle.crc(d.tobytes()), n


def test_update_strided_device_views(gpu, oracle):
    """update() over non-contiguous device views (every other byte, a column of a 2-D tensor, a
    transposed int32 tensor): checksummed over the view's elements in order, as its contiguous copy
    (ADVICE r3)."""
    rng = np.random.default_rng(31)
    d = rng.integers(0, 256, 1 << 18, dtype=np.uint8)
    t = torch.from_numpy(d).to(gpu)
    assert tk.crc32().update(t[::2]).finalize() == oracle.crc(d[::2].tobytes())
    m = t.view(512, 512)
    assert tk.crc32().update(m[:, 7]).finalize() == oracle.crc(np.ascontiguousarray(d.reshape(512, 512)[:, 7]).tobytes())
    w = t.view(torch.int32).view(256, 256).t()
    want = np.ascontiguousarray(d.view(np.int32).reshape(256, 256).T).tobytes()
    assert tk.crc32().update(w).finalize() == oracle.crc(want)
    assert tk.crc32c().update(t[1::3]).finalize() == oracle.crc_c(d[1::3].tobytes())


def test_update_on_side_stream(gpu, oracle):
    """update(tensor, stream=s) with s not the current stream: the kernel on s must see bytes the
    current stream has just written, and the result must be read after the kernel on s."""
    s = torch.cuda.Stream(device=gpu)
    base = torch.arange(1 << 24, dtype=torch.int64, device=gpu)
    for k in range(4):
        x = ((base * (2 * k + 1)) >> 3).to(torch.uint8)  # written on the current stream, just before
        got = tk.crc32().update(x, stream=s).finalize()
        assert got == oracle.crc(x.cpu().numpy().tobytes()), k


def test_batch_on_side_stream(gpu, oracle):
    """crc32_batch_uniform / crc32_batch on a side stream, with the output allocated by the call:
    ready once that stream is synchronised."""
    s = torch.cuda.Stream(device=gpu)
    n, blen = 3000, 4096
    data = torch.empty(n * blen, dtype=torch.uint8, device=gpu)
    tk.fill_synthetic_uniform(data, blen, n, first_block=11)
    s.wait_stream(torch.cuda.current_stream())
    out = tk.crc32_batch_uniform(data, blen, n, stream=s)
    offs = torch.arange(n, dtype=torch.int64, device=gpu) * blen
    lens = torch.full((n,), blen, dtype=torch.int32, device=gpu)
    s.wait_stream(torch.cuda.current_stream())
    out2 = tk.crc32_batch(data, offs, lens, stream=s)
    s.synchronize()
    want = oracle.synthetic(1, 11, n, blen)
    assert np.array_equal(u32(out), want) and np.array_equal(u32(out2), want)


def test_batch_on_side_stream_orders_itself(gpu, oracle):
    """No caller-side wait_stream: the batch entry points order the side stream after the current
    stream's prior work themselves, so bytes written there just before (and an `out` block the
    caching allocator reuses) are seen by the kernels on the side stream."""
    s = torch.cuda.Stream(device=gpu)
    n, blen = 2000, 4096
    base = torch.arange(n * blen // 8, dtype=torch.int64, device=gpu)
    for k in range(3):
        data = ((base * (2 * k + 3)) ^ (base >> 5)).view(torch.uint8)  # written on the current stream
        out = tk.crc32_batch_uniform(data, blen, n, stream=s)
        offs = torch.arange(n, dtype=torch.int64, device=gpu) * blen + 1
        lens = torch.full((n,), blen - 1, dtype=torch.int32, device=gpu)
        out2 = tk.crc32_batch(data, offs, lens, stream=s)
        s.synchronize()
        host = data.cpu().numpy()
        assert np.array_equal(u32(out), oracle.batch(host, np.arange(n) * blen, np.full(n, blen))), k
        assert np.array_equal(u32(out2), oracle.batch(host, offs.cpu().numpy(), lens.cpu().numpy())), k
        del out, out2  # freed blocks go back to the pool for the next round's allocations


def test_batch_argument_checks(gpu):
    data = torch.zeros(1 << 16, dtype=torch.uint8, device=gpu)
    offs = torch.zeros(4, dtype=torch.int64, device=gpu)
    lens = torch.ones(4, dtype=torch.int32, device=gpu)
    with pytest.raises(ValueError):
        tk.crc32_batch(data, offs, lens, out=torch.empty(3, dtype=torch.int32, device=gpu))  # short out
    with pytest.raises(ValueError):
        tk.crc32_batch(data, offs, lens, init_raw=torch.empty(2, dtype=torch.int32, device=gpu))
    with pytest.raises(ValueError):
        tk.crc32_batch(data, offs.cpu(), lens)
    with pytest.raises(ValueError):
        tk.crc32_batch_uniform(data, 4096, 16, out=torch.empty(16, dtype=torch.int64, device=gpu))


def test_update_chaining_raw_state(gpu, oracle):
    rng = np.random.default_rng(2)
    d = rng.integers(0, 256, 50000, dtype=np.uint8).tobytes()
    c = tk.crc32()
    for a, b in ((0, 1), (1, 3), (3, 4100), (4100, 4101), (4101, 50000)):
        c.update(d[a:b])
    assert c.finalize() == oracle.crc(d)


def test_update_latency_path_every_length(gpu, oracle):
    """Host spans of up to 16 KiB take the one-workgroup latency kernel (crc_span): every length
    0..300, then a sweep to 16 KiB and just past it (the staged path), from random raw registers,
    for both polynomials, each against the oracle (crc32.cpp:9-16 restated)."""
    rng = np.random.default_rng(21)
    buf = rng.integers(0, 256, (16 << 10) + 64, dtype=np.uint8).tobytes()
    lens = list(range(301)) + list(range(301, 16 << 10, 97)) + [4095, 4096, 4097, (16 << 10) - 1, 16 << 10,
                                                               (16 << 10) + 1, (16 << 10) + 63]
    for n in lens:
        raw = int(rng.integers(0, 2**32))
        c = tk.crc32()
        c._crc = raw
        assert c.update(buf[:n]).raw == oracle.update(raw, buf[:n]), n
    for n in (0, 1, 5, 36, 1000, 4097, 16 << 10):
        raw = int(rng.integers(0, 2**32))
        c = tk.crc32c()
        c._crc = raw
        assert c.update(buf[:n]).raw == oracle.update_c(raw, buf[:n]), n


def test_odd_prefixes(gpu, oracle):
    g = golden("odd.json")
    buf = oracle.fill(g["seed"], g["block"], 0, 1 << 20)
    t = torch.from_numpy(buf).to(gpu)
    lens = [p["len"] for p in g["prefixes"]]
    offs = torch.zeros(len(lens), dtype=torch.int64, device=gpu)
    ln = torch.tensor(lens, dtype=torch.int32, device=gpu)
    got = u32(tk.crc32_batch(t, offs, ln))
    assert [int(x) for x in got] == [p["crc"] for p in g["prefixes"]]
    for p in g["prefixes"]:
        assert tk.crc32().update(buf[:p["len"]].tobytes()).finalize() == p["crc"]


# ---- WAL call sites (wal.cpp:54-58, 89-96; wal_test.cpp, engine_test.cpp:437-459) ----------------

def test_wal_records_stamped_identically(gpu):
    """The stamp equals the reference encoder's bytes for every golden record, including
    {put,7,"test","data",0}, whose stored CRC wal_test.cpp:507-541 recomputes over [8, size)."""
    recs = golden("wal.json")["records"]
    unstamped = [tk.wal.encode_unstamped(r["op"], r["seq"], r["key"].encode(), r["value"].encode(),
                                         r["tombstone"]) for r in recs]
    stamped = tk.wal.stamp(unstamped)
    for r, s in zip(recs, stamped):
        assert s.hex() == r["hex"]
        assert struct.unpack_from("<I", s, 4)[0] == r["crc"]


def test_wal_verify_and_first_corruption(gpu):
    recs = [bytes.fromhex(r["hex"]) for r in golden("wal.json")["records"]]
    image = b"".join(recs)
    assert tk.wal.verify(image) == ("ok", len(recs), len(image))
    assert tk.wal.verify(b"") == ("ok", 0, 0)
    # flip the CRC byte of record 1 (wal_test.cpp:809-850): record 0 good, parked at record 1
    bad = bytearray(image)
    bad[len(recs[0]) + 4] ^= 0xFF
    assert tk.wal.verify(bytes(bad)) == ("corrupted", 1, len(recs[0]))
    # payload corruption of record 0 (wal_test.cpp:245-263)
    bad = bytearray(image)
    bad[10] ^= 0xFF
    assert tk.wal.verify(bytes(bad)) == ("corrupted", 0, 0)
    # truncated tail (wal.cpp:68-70 / 82-87)
    st, good, stop = tk.wal.verify(image[:-3])
    assert st == "corrupted" and good == len(recs) - 1


def test_wal_single_record_crc_byte_flip(gpu):
    """wal_test.cpp:341-364: {put,1,"k","v",0} with its first CRC byte inverted fails, and the view
    stays where it was (no good records, stop at byte 0)."""
    rec = bytearray(bytes.fromhex(golden("wal.json")["records"][2]["hex"]))
    rec[4] = ~rec[4] & 0xFF
    assert tk.wal.verify(bytes(rec)) == ("corrupted", 0, 0)
    assert tk.wal.verify(bytes(rec) + bytes.fromhex(golden("wal.json")["records"][0]["hex"])) == ("corrupted", 0, 0)


def test_wal_key_value_overflow_detected_after_crc(gpu):
    rec = bytearray(bytes.fromhex(golden("wal.json")["records"][2]["hex"]))  # {put,1,"k","v"}
    struct.pack_into("<I", rec, 18, 9999)  # wal_test.cpp:265-294: bogus key_len, CRC recomputed
    rec[4:8] = struct.pack("<I", tk.crc32().update(bytes(rec[8:])).finalize())
    assert tk.wal.verify(bytes(rec)) == ("corrupted", 0, 0)


def test_wal_many_records(gpu, oracle):
    rng = np.random.default_rng(9)
    recs = []
    for i in range(3000):
        k = rng.integers(0, 256, rng.integers(0, 40), dtype=np.uint8).tobytes()
        v = rng.integers(0, 256, rng.integers(0, 300), dtype=np.uint8).tobytes()
        recs.append(tk.wal.encode_unstamped(i % 2, i, k, v, i % 2))
    stamped = tk.wal.stamp(recs)
    for s in stamped[:200]:
        assert struct.unpack_from("<I", s, 4)[0] == oracle.crc(s[8:])
    image = b"".join(stamped)
    assert tk.wal.verify(image) == ("ok", 3000, len(image))


def big_wal(rng, n_rec, giant_at=None, giant_len=0):
    """A WAL image of n_rec records laid out as wal.cpp:19-61 (numpy, unstamped); optionally one
    giant value at record giant_at. Returns (image, offsets, sizes)."""
    klen = rng.integers(0, 40, n_rec).astype(np.uint64)
    vlen = np.minimum(rng.zipf(1.6, n_rec) * 64, 16000).astype(np.uint64)
    if giant_at is not None:
        vlen[giant_at] = giant_len
    size = 26 + klen + vlen
    offs = np.zeros(n_rec, np.uint64)
    offs[1:] = np.cumsum(size[:-1])
    img = rng.integers(0, 256, int(size.sum()), dtype=np.uint8)
    hdr = np.zeros((n_rec, 26), np.uint8)
    hdr[:, 0:4] = (size - 8).astype("<u4").view(np.uint8).reshape(-1, 4)
    hdr[:, 9:17] = np.arange(n_rec, dtype="<u8").view(np.uint8).reshape(-1, 8)
    hdr[:, 18:22] = klen.astype("<u4").view(np.uint8).reshape(-1, 4)
    hdr[:, 22:26] = vlen.astype("<u4").view(np.uint8).reshape(-1, 4)
    img[offs.astype(np.int64)[:, None] + np.arange(26)] = hdr
    return img, offs, size.astype(np.uint32)


@pytest.mark.parametrize("pinned", [False, True])
def test_wal_verify_large_image_phases(gpu, oracle, pinned):
    """A >= 64 MiB WAL is walked and checksummed in phases (the CRC batch of a phase overlaps the
    walk of the next): results, first-corruption position and truncation behave as one pass."""
    import ctypes
    rng = np.random.default_rng(41)
    img, offs, size = big_wal(rng, 120000, giant_at=50000, giant_len=30 << 20)
    lib = tk.load_library()
    keep = None
    if pinned:
        keep = torch.from_numpy(img).pin_memory()
        img = keep.numpy()
    tk.check(lib.tkv_wal_stamp(ctypes.c_void_p(img.ctypes.data), ctypes.c_void_p(offs.ctypes.data),
                               ctypes.c_void_p(size.ctypes.data), offs.size))
    for i in (0, 49999, 50000, 50001, 119999):  # stamps equal the oracle's (wal.cpp:54-58)
        o, n = int(offs[i]), int(size[i])
        assert int(img[o + 4:o + 8].view("<u4")[0]) == oracle.crc(img[o + 8:o + n].tobytes())
    assert img.size >= 64 << 20
    good, stop = ctypes.c_uint64(0), ctypes.c_uint64(0)

    def verify(buf, nbytes):
        rc = lib.tkv_wal_verify(ctypes.c_void_p(buf.ctypes.data), nbytes, ctypes.byref(good), ctypes.byref(stop))
        return rc, good.value, stop.value

    assert verify(img, img.size) == (0, offs.size, img.size)
    for bad in (3, 50000, 90001):  # first phase, the giant record, a late phase
        o = int(offs[bad]) + 26
        img[o] ^= 0x10
        rc, g, st = verify(img, img.size)
        img[o] ^= 0x10
        assert rc != 0 and (g, st) == (bad, int(offs[bad]))
    rc, g, st = verify(img, img.size - 5)  # truncated tail: the last record does not fit
    assert rc != 0 and (g, st) == (offs.size - 1, int(offs[-1]))


# ---- uniform batches ---------------------------------------------------------------------------

@pytest.mark.parametrize("blen,n", [(4096, 5000), (65536, 300), (4096, 7), (16, 100000), (1000, 9000),
                                    (4100, 4097), (12288, 513), (1, 4096), (0, 10), (3, 20000)])
def test_uniform_vs_oracle(gpu, oracle, blen, n):
    stride = max(blen, 8) + (8 - max(blen, 8) % 8) % 8
    data = torch.empty(n * stride + 16, dtype=torch.uint8, device=gpu)
    if blen % 8 == 0 and blen:
        tk.fill_synthetic_uniform(data, blen, n, first_block=3, stride=stride)
        want = oracle.synthetic(1, 3, n, blen)
        got = u32(tk.crc32_batch_uniform(data, blen, n, stride=stride))
        assert np.array_equal(got, want)
    host = np.random.default_rng(blen).integers(0, 256, n * stride + 16, dtype=np.uint8)
    data.copy_(torch.from_numpy(host))
    want = oracle.batch(host, np.arange(n) * stride, np.full(n, blen))
    got = u32(tk.crc32_batch_uniform(data, blen, n, stride=stride))
    assert np.array_equal(got, want)
    # same blocks at an odd (unaligned) base address
    got = u32(tk.crc32_batch_uniform(data, blen, n, stride=stride, offset=5)) if (n - 1) * stride + blen + 5 <= data.numel() else None
    if got is not None:
        want = oracle.batch(host, np.arange(n) * stride + 5, np.full(n, blen))
        assert np.array_equal(got, want)


def test_uniform_per_block_init(gpu, oracle):
    n, blen = 2000, 4096
    host = np.random.default_rng(4).integers(0, 256, n * blen, dtype=np.uint8)
    init = np.random.default_rng(5).integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    got = u32(tk.crc32_batch_uniform(torch.from_numpy(host).to(gpu), blen, n,
                                     init_raw=torch.from_numpy(init.view(np.int32)).to(gpu)))
    want = oracle.batch(host, np.arange(n) * blen, np.full(n, blen), init)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("blen,n", [(4096, 4096), (8192, 4500), (12288, 9000), (65536, 4097)])
def test_packed_fast_path(gpu, oracle, blen, n):
    """len % 4 KiB == 0, stride == len, aligned, n >= waves: the crc_packed kernel."""
    host = np.random.default_rng(blen + n).integers(0, 256, n * blen, dtype=np.uint8)
    d = torch.from_numpy(host).to(gpu)
    want = oracle.batch(host, np.arange(n) * blen, np.full(n, blen))
    assert np.array_equal(u32(tk.crc32_batch_uniform(d, blen, n)), want)
    init = np.random.default_rng(n).integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    got = u32(tk.crc32_batch_uniform(d, blen, n, init_raw=torch.from_numpy(init.view(np.int32)).to(gpu)))
    assert np.array_equal(got, oracle.batch(host, np.arange(n) * blen, np.full(n, blen), init))


def test_single_huge_block_split_across_waves(gpu, oracle):
    n = (64 << 20) + 77  # one block, rows spread over every wave, joined by crc_fixup
    host = np.random.default_rng(6).integers(0, 256, n, dtype=np.uint8)
    got = u32(tk.crc32_batch_uniform(torch.from_numpy(host).to(gpu), n, 1))
    assert int(got[0]) == oracle.crc(host.tobytes())


# ---- irregular batches ---------------------------------------------------------------------------

def irregular_case(rng, nblocks, maxlen, packed=True, overlap=False):
    lens = rng.integers(0, maxlen + 1, nblocks)
    lens[rng.integers(0, nblocks, max(1, nblocks // 50))] = rng.integers(0, 4, max(1, nblocks // 50))
    if packed:
        offs = np.concatenate([[0], np.cumsum(lens[:-1])]) + 3
    else:
        offs = rng.integers(0, int(lens.sum()) + 1, nblocks)
    size = int((offs + lens).max()) + 32
    host = rng.integers(0, 256, size, dtype=np.uint8)
    return host, offs.astype(np.int64), lens.astype(np.int32)


@pytest.mark.parametrize("nblocks,maxlen,packed", [(1, 100, True), (10, 5000, True), (5000, 300, True),
                                                   (3000, 20000, False), (200, 300000, True),
                                                   (70000, 64, True)])
def test_irregular_vs_oracle(gpu, oracle, nblocks, maxlen, packed):
    rng = np.random.default_rng(nblocks + maxlen)
    host, offs, lens = irregular_case(rng, nblocks, maxlen, packed)
    init = rng.integers(0, 2**32, nblocks, dtype=np.uint64).astype(np.uint32)
    d = torch.from_numpy(host).to(gpu)
    o = torch.from_numpy(offs).to(gpu)
    ln = torch.from_numpy(lens).to(gpu)
    got = u32(tk.crc32_batch(d, o, ln))
    assert np.array_equal(got, oracle.batch(host, offs, lens))
    got = u32(tk.crc32_batch(d, o, ln, init_raw=torch.from_numpy(init.view(np.int32)).to(gpu)))
    assert np.array_equal(got, oracle.batch(host, offs, lens, init))


@pytest.mark.parametrize("mix", ["all_small", "boundary", "alternating", "small_at_buffer_edges"])
def test_small_block_split(gpu, oracle, mix):
    """The prepass splits blocks at kSmallMax = 1024 bytes: small ones are folded four to a wave by
    crc_small, large ones by the row kernel on a compacted list; results land at batch indices."""
    rng = np.random.default_rng(len(mix))
    if mix == "all_small":
        lens = rng.integers(0, 1025, 20000)
    elif mix == "boundary":
        lens = np.tile(np.array([0, 1, 3, 15, 16, 17, 1023, 1024, 1025, 1026, 2047, 4095, 4096, 4097]), 300)
    elif mix == "alternating":
        lens = np.where(np.arange(6001) % 2 == 0, rng.integers(0, 1025, 6001), rng.integers(1025, 30000, 6001))
    else:
        lens = rng.integers(0, 1025, 3001)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
    if mix == "alternating":
        offs += rng.integers(0, 16, lens.size).cumsum()  # gaps: any alignment
    size = int((offs + lens).max()) + (0 if mix == "small_at_buffer_edges" else 40)
    host = rng.integers(0, 256, max(size, 1), dtype=np.uint8)
    d = torch.from_numpy(host).to(gpu)
    o = torch.from_numpy(offs).to(gpu)
    ln = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    want = oracle.batch(host, offs, lens.astype(np.int32))
    assert np.array_equal(u32(tk.crc32_batch(d, o, ln)), want)
    init = rng.integers(0, 2**32, lens.size, dtype=np.uint64).astype(np.uint32)
    got = u32(tk.crc32_batch(d, o, ln, init_raw=torch.from_numpy(init.view(np.int32)).to(gpu)))
    assert np.array_equal(got, oracle.batch(host, offs, lens.astype(np.int32), init))
    # a second, smaller batch on the same stream reuses the scratch of the first
    m = max(1, lens.size // 7)
    assert np.array_equal(u32(tk.crc32_batch(d, o[:m].contiguous(), ln[:m].contiguous())), want[:m])


def test_irregular_more_than_fused_tiles(gpu, oracle):
    """Batches of more than 1024 scan tiles (4096 blocks each) take the unfused prepass: tile scan,
    single-workgroup scan of the tile sums, then the scatter (launch_prepass, tkv_crc32_kernels.hip).
    4 M + 4097 mostly tiny blocks with a large one every 997 blocks, so both the small-block phase
    and the row kernel's wave partition see tiles past the fused limit."""
    rng = np.random.default_rng(4097)
    n = 4096 * 1024 + 4097
    lens = rng.integers(0, 65, n).astype(np.int64)
    lens[::997] = rng.integers(1025, 9000, lens[::997].size)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
    host = rng.integers(0, 256, int(lens.sum()) + 16, dtype=np.uint8)
    d = torch.from_numpy(host).to(gpu)
    o = torch.from_numpy(offs).to(gpu)
    ln = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    want = oracle.batch(host, offs, lens)
    assert np.array_equal(u32(tk.crc32_batch(d, o, ln)), want)
    # the same stream's scratch then serves a fused-size batch
    m = 4096 * 1024 - 1
    assert np.array_equal(u32(tk.crc32_batch(d, o[:m].contiguous(), ln[:m].contiguous())), want[:m])


def test_irregular_zipf_sample(gpu, oracle):
    """First 4096 blocks of cfg4 (Zipf 256 B - 1 MiB), packed back to back, unaligned starts."""
    c = golden("synthetic.json")["cfg4"]
    lens = oracle.zipf_lengths(1, 0, 4096)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
    d = torch.empty(int(lens.sum()) + 64, dtype=torch.uint8, device=gpu)
    o = torch.from_numpy(offs).to(gpu)
    ln = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    tk.fill_synthetic_blocks(d, o, ln, first_block=0)
    got = u32(tk.crc32_batch(d, o, ln))
    assert [int(x) for x in got[:256]] == c["first"]
    assert np.array_equal(got, oracle.synthetic_lens(1, 0, lens))


def test_corruption_always_detected(gpu):
    n, blen = 1024, 4096
    host = np.random.default_rng(8).integers(0, 256, n * blen, dtype=np.uint8)
    d = torch.from_numpy(host).to(gpu)
    clean = u32(tk.crc32_batch_uniform(d, blen, n))
    rng = np.random.default_rng(9)
    pos = rng.integers(0, n * blen, 256)
    bits = rng.integers(0, 8, 256)
    for p, b in zip(pos, bits):
        host[p] ^= np.uint8(1 << int(b))
    d2 = torch.from_numpy(host).to(gpu)
    dirty = u32(tk.crc32_batch_uniform(d2, blen, n))
    hit = np.zeros(n, bool)
    hit[np.unique(pos // blen)] = True
    assert np.array_equal(clean != dirty, hit)  # every single-bit-flipped block differs, no others


# ---- host pipeline and multi-device host API ----------------------------------------------------

def test_host_batch(gpu, oracle):
    rng = np.random.default_rng(12)
    host, offs, lens = irregular_case(rng, 20000, 20000, packed=False)
    got = tk.crc32_batch_host(host, offs, lens)
    assert np.array_equal(got, oracle.batch(host, offs, lens))
    got = tk.crc32_batch_host(host, offs, lens, devices=[0])
    assert np.array_equal(got, oracle.batch(host, offs, lens))


@pytest.mark.parametrize("n,maxlen", [(1, 36), (2, 5), (17, 4096), (256, 200), (256, 256), (257, 40),
                                      (3, 16 << 10), (4, 16 << 10), (40, 2000)])
def test_host_small_batches(gpu, oracle, n, maxlen):
    """Host batches of at most 256 spans of at most 16 KiB and 64 KiB in all (a WAL group commit)
    take the one-launch latency path (crc_span, a workgroup per span); 257 spans, or more than
    64 KiB in all, take the staged pipeline. Both against the oracle, with and without per-block
    initial registers, both polynomials, lengths from 0, unaligned offsets."""
    rng = np.random.default_rng(n * 7 + maxlen)
    host = rng.integers(0, 256, n * maxlen + 64, dtype=np.uint8)
    lens = rng.integers(0, maxlen + 1, n).astype(np.uint32)
    lens[0] = maxlen
    offs = np.array([int(rng.integers(0, host.size - int(ln))) for ln in lens], np.uint64)
    assert np.array_equal(tk.crc32_batch_host(host, offs, lens), oracle.batch(host, offs, lens))
    init = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    assert np.array_equal(tk.crc32_batch_host(host, offs, lens, init_raw=init), oracle.batch(host, offs, lens, init))
    got_c = tk.crc32_batch_host(host, offs, lens, algo="crc32c")
    want_c = [oracle.crc_c(host[int(o):int(o) + int(ln)].tobytes()) for o, ln in zip(offs, lens)]
    assert [int(x) for x in got_c] == want_c


def test_host_batch_block_larger_than_slab(gpu, oracle):
    n = (300 << 20) + 5
    host = np.random.default_rng(13).integers(0, 256, n, dtype=np.uint8)
    got = tk.crc32_batch_host(host, [0, 7, 1 << 20], [n, 100, 4096])
    want = [oracle.crc(host.tobytes()), oracle.crc(host[7:107].tobytes()), oracle.crc(host[1 << 20:(1 << 20) + 4096].tobytes())]
    assert [int(x) for x in got] == want


@pytest.mark.parametrize("stride", [None, 4096])
def test_host_batch_dense_run_longer_than_slab(gpu, oracle, stride):
    """Pageable blocks 8 bytes apart (WAL payloads) whose covering range exceeds a 256 MiB staging
    slab: each slab ends at the block that would push its range past 256 MiB and goes over as one
    range. Random lengths, and 4088-byte blocks on a 4096-byte stride, whose first slab's range
    ends 8 bytes short of 256 MiB. Against the oracle."""
    rng = np.random.default_rng(29)
    if stride is None:
        lens = rng.integers(1, 16 << 10, 40_000).astype(np.uint32)
    else:
        lens = np.full(70_000, stride - 8, np.uint32)
    offs = np.concatenate([[8], np.cumsum(lens.astype(np.uint64) + 8)[:-1] + 8]).astype(np.uint64)
    host = rng.integers(0, 256, int(offs[-1]) + int(lens[-1]), dtype=np.uint8)
    assert host.size > (256 << 20)
    assert np.array_equal(tk.crc32_batch_host(host, offs, lens), oracle.batch(host, offs, lens))


@pytest.mark.parametrize("ndev", [2, 3, 4])
def test_host_multi_splits_large_blocks(gpu, oracle, ndev):
    """Blocks of >= 1 MiB that straddle a device share are cut at the share boundary and their
    pieces combine on the host: a single 9 MiB block over ndev devices, and a mixed batch
    with per-block initial registers, both equal to the oracle. Device 0 stands in for every device."""
    rng = np.random.default_rng(41 + ndev)
    n = 9 << 20
    host = rng.integers(0, 256, n + 4096, dtype=np.uint8)
    got = tk.crc32_batch_host(host, [3], [n], devices=[0] * ndev)
    assert int(got[0]) == oracle.crc(host[3:3 + n].tobytes())
    offs = np.array([0, 5, (3 << 20) + 9, 17, (5 << 20) + 1, 11], np.uint64)
    lens = np.array([(3 << 20) + 1, 0, (2 << 20) + 77, 100, 1 << 20, (4 << 20) - 3], np.uint32)
    init = rng.integers(0, 1 << 32, offs.size, dtype=np.uint64).astype(np.uint32)
    for algo in ("crc32", "crc32c"):
        got = tk.crc32_batch_host(host, offs, lens, init_raw=init, devices=[0] * ndev, algo=algo)
        want = tk.crc32_batch_host(host, offs, lens, init_raw=init, algo=algo)
        assert np.array_equal(got, want)
    assert np.array_equal(tk.crc32_batch_host(host, offs, lens, init_raw=init, devices=[0] * ndev),
                          oracle.batch(host, offs, lens, init))


def pinned_copy(a):
    """numpy view of a pinned (hipHostMalloc) copy of ``a``: the kernels can read it in place."""
    t = torch.empty(a.size, dtype=torch.uint8).pin_memory()
    t.numpy()[:] = a
    return t, t.numpy()


@pytest.mark.parametrize("packed", [False, True])
def test_host_batch_pinned_zero_copy(gpu, oracle, packed):
    """Pinned sources are read in place by the kernels (no staging copy); results equal the staged
    pipeline's and the oracle's, with and without per-block initial registers."""
    rng = np.random.default_rng(21)
    host, offs, lens = irregular_case(rng, 5000, 70000, packed=packed)
    keep, pin = pinned_copy(host)
    want = oracle.batch(host, offs, lens)
    lib = tk.load_library()
    assert lib.tkv_debug_set_host_mapped(1) == 1
    got = tk.crc32_batch_host(pin, offs, lens)
    assert np.array_equal(got, want)
    init = rng.integers(0, 1 << 32, offs.size, dtype=np.uint64).astype(np.uint32)
    want_i = oracle.batch(host, offs, lens, init)
    assert np.array_equal(tk.crc32_batch_host(pin, offs, lens, init_raw=init), want_i)
    assert lib.tkv_debug_set_host_mapped(0) == 1
    try:
        assert np.array_equal(tk.crc32_batch_host(pin, offs, lens, init_raw=init), want_i)
    finally:
        lib.tkv_debug_set_host_mapped(1)
    assert np.array_equal(tk.crc32_batch_host(pin, offs, lens, devices=[0, 0]), want)
    assert np.array_equal(tk.crc32_batch_host(pin, offs, lens, algo="crc32c"),
                          tk.crc32_batch_host(host, offs, lens, algo="crc32c"))


def test_host_batch_pinned_uniform_and_huge(gpu, oracle):
    """Uniform contiguous pinned batches take the packed kernel in place; a block larger than a
    staging slab is one block of the in-place irregular batch (no chaining)."""
    n, blen = 5000, 65536  # 312.5 MiB: room for a block larger than a 256 MiB staging slab
    dev = torch.empty(n * blen, dtype=torch.uint8, device="cuda")
    tk.fill_synthetic_uniform(dev, blen, n, first_block=5)
    keep = dev.cpu().pin_memory()
    pin = keep.numpy()
    want = np.zeros(n, np.uint32)
    oracle.lib.oracle_crc_synthetic(1, 5, n, blen, want.ctypes.data)
    offs = np.arange(n, dtype=np.uint64) * blen
    assert np.array_equal(tk.crc32_batch_host(pin, offs, np.full(n, blen, np.uint32)), want)
    big = (300 << 20) + 5
    assert big <= pin.size
    got = tk.crc32_batch_host(pin, [0, 7, 1 << 20], [big, 100, 4096])
    assert [int(x) for x in got] == [oracle.crc(pin[:big].tobytes()), oracle.crc(pin[7:107].tobytes()),
                                     oracle.crc(pin[1 << 20:(1 << 20) + 4096].tobytes())]


def test_host_batch_pinned_sees_host_writes_between_calls(gpu, oracle):
    """In-place reads of pinned memory see every host write made before the call (no stale device
    cache lines from an earlier call over the same buffer)."""
    rng = np.random.default_rng(23)
    keep, pin = pinned_copy(rng.integers(0, 256, 8 << 20, dtype=np.uint8))
    offs = np.arange(0, 8 << 20, 65536, dtype=np.uint64)
    lens = np.full(offs.size, 65536, np.uint32)
    for it in range(6):
        got = tk.crc32_batch_host(pin, offs, lens)
        assert np.array_equal(got, oracle.batch(pin, offs, lens)), it
        pos = rng.integers(0, pin.size, 1000)
        pin[pos] ^= rng.integers(1, 256, pos.size, dtype=np.uint8)  # host writes, then the next call


def test_host_batch_registered_range_checked(gpu, oracle):
    """Part of a pageable buffer pinned with hipHostRegister: a batch inside the registered range
    may be read in place, one that leaves it must be staged (never read by the kernels past the
    registration) - both give the oracle's CRCs."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    rng = np.random.default_rng(22)
    big = rng.integers(0, 256, 8 << 20, dtype=np.uint8)
    page = 1 << 16
    start = (-big.ctypes.data) % page
    reg = big[start:start + (4 << 20)]  # registered window, page aligned
    assert hip.hipHostRegister(reg.ctypes.data, reg.size, 0) == 0
    try:
        inside_o = np.array([0, 4096, (4 << 20) - 65536], np.uint64)
        inside_l = np.array([4096, 100000, 65536], np.uint32)
        assert np.array_equal(tk.crc32_batch_host(reg, inside_o, inside_l), oracle.batch(reg, inside_o, inside_l))
        tail = big[start:]  # same base, but the last block runs past the registered window
        out_o = np.array([0, (4 << 20) - 4096], np.uint64)
        out_l = np.array([4096, 2 << 20], np.uint32)
        assert np.array_equal(tk.crc32_batch_host(tail, out_o, out_l), oracle.batch(tail, out_o, out_l))
    finally:
        hip.hipHostUnregister(reg.ctypes.data)


# ---- full-size BASELINE configs through golden aggregates ----------------------------------------

def aggregates(crcs):
    return int(np.bitwise_xor.reduce(crcs)), int(crcs.astype(np.uint64).sum() & 0xFFFFFFFF)


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3", "cfg5"])
def test_full_size_uniform_configs(gpu, cfg):
    """cfg5 (4 M x 64 KiB = 256 GiB, BASELINE's 8-GPU config) runs here as its eight 32 GiB
    per-GPU shards in turn on one device; its aggregates pin the sharded result."""
    c = golden("synthetic.json")[cfg]
    n, blen = c["nblocks"], c["len"]
    got = np.zeros(n, np.uint32)
    chunk = min(n, ((32 if cfg == "cfg5" else 4) << 30) // blen)  # device data per pass
    data = torch.empty(chunk * blen, dtype=torch.uint8, device=gpu)
    shards = {sh["first_block"]: sh for sh in golden("synthetic.json")["shards"][cfg]} if cfg == "cfg5" else {}
    for first in range(0, n, chunk):
        m = min(chunk, n - first)
        tk.fill_synthetic_uniform(data, blen, m, first_block=first)
        got[first:first + m] = u32(tk.crc32_batch_uniform(data, blen, m))
        if first in shards:  # cfg5: each 32 GiB pass is one rank's shard
            assert aggregates(got[first:first + m]) == (shards[first]["xor"], shards[first]["sum32"]), first
    if "first" in c:
        assert [int(x) for x in got[:len(c["first"])]] == c["first"]
        assert int(got[-1]) == c["last"]
    assert aggregates(got) == (c["xor"], c["sum32"])


def test_full_size_zipf_config(gpu, oracle):
    c = golden("synthetic.json")["cfg4"]
    lens = oracle.zipf_lengths(1, 0, c["nblocks"])
    offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
    d = torch.empty(int(lens.sum()) + 64, dtype=torch.uint8, device=gpu)
    o = torch.from_numpy(offs).to(gpu)
    ln = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    tk.fill_synthetic_blocks(d, o, ln, first_block=0)
    got = u32(tk.crc32_batch(d, o, ln))
    assert [int(x) for x in got[:256]] == c["first"]
    assert aggregates(got) == (c["xor"], c["sum32"])


@pytest.mark.parametrize("cfg", ["cfg2", "cfg3", "cfg4"])
def test_rank_shards_full_size(gpu, oracle, cfg):
    """The per-rank shards of an 8-GPU bench run (rank r: global blocks [r*n, (r+1)*n), bench.py
    rank_shard), each checksummed whole on this device and compared with its golden XOR/SUM32
    (tests/golden/make_golden.py --shards). Rank 0 is the single-GPU config, checked above; cfg5's
    eight shards are checked in test_full_size_uniform_configs."""
    g = golden("synthetic.json")
    for sh in g["shards"][cfg][1:]:
        first, n = sh["first_block"], sh["nblocks"]
        if cfg == "cfg4":
            lens = oracle.zipf_lengths(1, first, n)
            offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
            d = torch.empty(int(lens.sum()) + 64, dtype=torch.uint8, device=gpu)
            o = torch.from_numpy(offs).to(gpu)
            ln = torch.from_numpy(lens.astype(np.int32)).to(gpu)
            tk.fill_synthetic_blocks(d, o, ln, first_block=first)
            got = u32(tk.crc32_batch(d, o, ln))
            assert int(lens.sum()) == sh["total_bytes"]
        else:
            blen = g[cfg]["len"]
            d = torch.empty(n * blen, dtype=torch.uint8, device=gpu)
            tk.fill_synthetic_uniform(d, blen, n, first_block=first)
            got = u32(tk.crc32_batch_uniform(d, blen, n))
        del d
        assert aggregates(got) == (sh["xor"], sh["sum32"]), f"{cfg} shard at block {first}"


@pytest.mark.parametrize("blen", [16, 48, 64, 80, 128, 144, 256, 512, 1024, 1040, 2000, 2048, 2064, 3008, 4080])
def test_packed_small_blocks(gpu, oracle, blen):
    """Uniform batches of small blocks packed back to back (G-lane groups, each block right-aligned
    in a 64*G-byte slot, 64/G blocks per wave row): batches ending in a partial row,
    single blocks, and a batch large enough for every wave, against the oracle; raw registers
    through update_device."""
    rng = np.random.default_rng(blen)
    g = 1
    while 64 * g < blen:
        g *= 2
    bpr = 64 // g
    for n in (1, 2, bpr - 1, bpr, bpr + 1, 4096 * bpr + 3, 300_000 // max(1, blen // 64)):
        host = rng.integers(0, 256, n * blen + 64, dtype=np.uint8)
        d = torch.from_numpy(host).to(gpu)
        got = u32(tk.crc32_batch_uniform(d, blen, n))
        offs = np.arange(n, dtype=np.uint64) * blen
        want = oracle.batch(host, offs, np.full(n, blen, np.uint32))
        bad = np.flatnonzero(got != want)
        assert bad.size == 0, (n, bad[:5])
    c = tk.crc32().update(torch.from_numpy(host[:blen].copy()).to(gpu))
    assert c.finalize() == oracle.crc(host[:blen].tobytes())
