"""GPU parity of the lane-block kernels: blocks of at most kLaneMax = 64 bytes, each
folded whole by one lane from its own initial register.

Uniform batches take crc_lanes (any stride, alignment and per-block init); irregular batches fold
their lane blocks in crc_stream's launch (general path) while the prepass lists only the rest. The
shapes are the reference's WAL records: 26 + |k| + |v| bytes (/root/reference/src/engine/wal.cpp:25,
kMetadataSize in wal.hpp:21-27), stamped one per put (wal.cpp:54-57), whose payloads lie 8 header
bytes apart in an image. Everything is compared block by block with the oracle.
"""
import ctypes

import numpy as np
import pytest

import tinykvpp_amd as tk
from conftest import lists_expected, phases_expected

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

WAL_SIZES = (26, 28, 33, 36, 59)


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def mode():
    """Path the last irregular batch on the current stream took: 0 general, 1 stream mode."""
    return tk.load_library().tkv_debug_irregular_mode(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))


def i32(a):
    return torch.from_numpy(np.ascontiguousarray(a, np.uint32).view(np.int32))


def oracle_c(oracle, host, offs, lens, init=None):
    """CRC-32C finalize() values of the blocks (the oracle's restatement, one call per block)."""
    out = np.zeros(len(offs), np.uint32)
    for i, (o, n) in enumerate(zip(offs, lens)):
        raw = 0xFFFFFFFF if init is None else int(init[i])
        out[i] = oracle.update_c(raw, host[int(o):int(o) + int(n)].tobytes()) ^ 0xFFFFFFFF
    return out


@pytest.fixture(scope="module")
def buf(gpu):
    rng = np.random.default_rng(64)
    host = rng.integers(0, 256, (64 << 20) + 4096, dtype=np.uint8)
    return host, torch.from_numpy(host).to(gpu)


@pytest.mark.parametrize("blen", list(range(0, 65)))
def test_uniform_every_length(gpu, oracle, buf, blen):
    """Every length 0..64 with strides equal to, past (a WAL header's 8 bytes) and below the length
    (overlapping blocks), base pointers at every alignment class, batches ending inside a 64-block
    step, and per-block initial registers."""
    host, d = buf
    rng = np.random.default_rng(1000 + blen)
    cases = [(blen, 0, 1), (blen, 0, 64), (blen + 8, 5, 65), (max(blen, 1) + 3, 13, 1000),
             (blen + 8, 4, 4097), (max(blen - 7, 0), 1, 300), (59, 7, 2000), (blen, 8, 70_001)]
    for stride, offset, n in cases:
        offs = offset + np.arange(n, dtype=np.int64) * stride
        lens = np.full(n, blen, np.int32)
        want = oracle.batch(host, offs, lens)
        got = u32(tk.crc32_batch_uniform(d, blen, n, stride=stride, offset=offset))
        bad = np.flatnonzero(got != want)
        assert bad.size == 0, (stride, offset, n, bad[:5])
        init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        got = u32(tk.crc32_batch_uniform(d, blen, n, stride=stride, offset=offset, init_raw=i32(init).to(gpu)))
        assert np.array_equal(got, oracle.batch(host, offs, lens, init)), (stride, offset, n)


@pytest.mark.parametrize("blen", WAL_SIZES + (64,))
def test_uniform_full_waves(gpu, oracle, buf, blen):
    """1 M WAL-record-sized blocks back to back (every wave of every workgroup busy), aligned and at
    an odd base."""
    host, d = buf
    n = 1 << 20
    for offset in (0, 3):
        offs = offset + np.arange(n, dtype=np.int64) * blen
        want = oracle.batch(host, offs, np.full(n, blen, np.int32))
        got = u32(tk.crc32_batch_uniform(d, blen, n, offset=offset))
        assert np.array_equal(got, want), offset


def test_uniform_crc32c(gpu, oracle, buf):
    host, d = buf
    for blen, stride, offset, n in ((36, 44, 0, 3000), (59, 59, 5, 1999), (0, 4, 0, 10), (64, 64, 16, 700)):
        offs = offset + np.arange(n, dtype=np.int64) * stride
        got = u32(tk.crc32_batch_uniform(d, blen, n, stride=stride, offset=offset, algo="crc32c"))
        assert np.array_equal(got, oracle_c(oracle, host, offs, np.full(n, blen))), (blen, stride)
        init = np.random.default_rng(n).integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        got = u32(tk.crc32_batch_uniform(d, blen, n, stride=stride, offset=offset, init_raw=i32(init).to(gpu),
                                         algo="crc32c"))
        assert np.array_equal(got, oracle_c(oracle, host, offs, np.full(n, blen), init)), (blen, stride)


def wal_payloads(rng, n, sizes, base):
    """Payload offsets/lengths of a WAL image: each record is an 8-byte header (length, CRC) followed
    by its payload, so consecutive payloads lie 8 bytes apart."""
    lens = rng.choice(np.asarray(sizes), n).astype(np.int64)
    starts = base + 8 + np.concatenate([[0], np.cumsum(lens[:-1] + 8)])
    return starts.astype(np.int64), lens.astype(np.int32)


@pytest.mark.parametrize("sizes", [(36,), WAL_SIZES, tuple(range(0, 65))])
@pytest.mark.parametrize("base", [0, 1, 6, 11])
def test_irregular_wal_payloads(gpu, oracle, buf, sizes, base):
    """A device batch of WAL payloads: lane blocks only, gapped, at every base alignment; the prepass
    takes the general path and crc_stream's launch folds every block."""
    host, d = buf
    rng = np.random.default_rng(len(sizes) * 16 + base)
    offs, lens = wal_payloads(rng, 120_000, sizes, base)
    o, ln = torch.from_numpy(offs).to(gpu), torch.from_numpy(lens).to(gpu)
    got = u32(tk.crc32_batch(d, o, ln))
    assert mode() == 0
    assert np.array_equal(got, oracle.batch(host, offs, lens))
    init = rng.integers(0, 2**32, offs.size, dtype=np.uint64).astype(np.uint32)
    got = u32(tk.crc32_batch(d, o, ln, init_raw=i32(init).to(gpu)))
    assert np.array_equal(got, oracle.batch(host, offs, lens, init))


@pytest.mark.parametrize("shape", ["shuffled", "late_shuffle", "late_long", "spread", "tiny_batch", "zero_lengths",
                                   "at_allocation_end", "crc32c"])
def test_irregular_one_pass_lanes(gpu, oracle, buf, shape):
    """crc_list_lanes, the one-pass kernel in front of the general path for irregular batches with the
    default register: steps of 64 blocks staged through an LDS window when they lie in
    4 KiB, per-lane granule loads for a later step that does not (blocks out of order, spread out),
    its packed mode from the step where a first step does not fit or a block is over 64 bytes (near
    the start or the end), every length 0-64, batches ending inside a step, empty blocks, blocks ending
    at the last byte of their allocation, and CRC-32C on the same kernel. Batches of at least 1 M blocks
    (the kernel's threshold) except the tiny one."""
    host, d = buf
    rng = np.random.default_rng(sum(map(ord, shape)))
    offs, lens = wal_payloads(rng, 1_100_003, tuple(range(0, 65)), 3)  # (>= 256 K blocks: the one-pass kernel runs)
    # the kernel's 64-block steps that start no wave's range (a wave whose first step does not fit one
    # window sends the whole batch to the general path), from the kernel's own wave count
    ts = (offs.size + 63) // 64
    nw = int(tk.load_library().tkv_debug_list_lanes_waves(offs.size))
    assert nw > 0
    later = np.setdiff1d(np.arange(ts - 1), np.arange(nw, dtype=np.int64) * ts // nw)
    if shape == "shuffled":
        p = rng.permutation(offs.size)
        offs, lens = offs[p], lens[p]
    elif shape == "late_shuffle":  # every wave's first step fits; a third of the later steps are out of order
        for st in later[rng.random(later.size) < 0.33]:
            p = st * 64 + rng.permutation(64)
            offs[st * 64:st * 64 + 64], lens[st * 64:st * 64 + 64] = offs[p], lens[p]
    elif shape == "late_long":
        lens[-5] = 65
    elif shape == "spread":  # every 97th later step's blocks far apart
        for st in later[::97]:
            offs[st * 64:st * 64 + 64] = rng.integers(0, host.size - 64, 64)
    elif shape == "tiny_batch":  # (below the one-pass kernel's threshold: the general path)
        offs, lens = offs[:37], lens[:37]
    elif shape == "zero_lengths":
        lens[rng.random(lens.size) < 0.3] = 0
    elif shape == "at_allocation_end":
        n = 1 << 20
        lens = rng.integers(0, 65, n).astype(np.int32)
        offs = (host.size - 64 * n + 64 * np.arange(n) + (64 - lens)).astype(np.int64)  # each ends a 64-byte slot
    o, ln = torch.from_numpy(offs).to(gpu), torch.from_numpy(lens).to(gpu)
    if shape == "crc32c":
        got = u32(tk.crc32_batch(d, o, ln, algo="crc32c"))
        sample = rng.choice(offs.size, 20_000, replace=False)
        assert np.array_equal(got[sample], oracle_c(oracle, host, offs[sample], lens[sample]))
        return
    got = u32(tk.crc32_batch(d, o, ln))
    # which path folded the batch: crc_list_lanes one lane per block (0), or with its packed mode in some
    # wave (1: a first step out of order, a block over 64 bytes); the general path alone below 256 K blocks (3)
    want_path = {"shuffled": 1, "late_long": 1, "tiny_batch": 3}.get(shape, 0)
    assert path() == want_path, shape
    assert phases() == 0, shape
    want = oracle.batch(host, offs, lens)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (shape, bad[:5])
    if shape == "at_allocation_end":  # a copy whose last byte is the allocation's last byte
        tail = d[host.size - 64 * n:].clone()
        got = u32(tk.crc32_batch(tail, torch.from_numpy(offs - (host.size - 64 * n)).to(gpu), ln))
        assert np.array_equal(got, want)


@pytest.mark.parametrize("mix", ["lane_small_large", "lane_then_large", "random_offsets", "lane_at_buffer_end"])
def test_irregular_mixed_classes(gpu, oracle, mix):
    """Lane blocks (<= 64 B), small blocks (<= 1 KiB) and large ones in one batch: each class goes to
    its own phase and every result lands at its batch index; CRC-32C on the same batch."""
    rng = np.random.default_rng(len(mix))
    n = 30_000
    if mix == "lane_small_large":
        lens = rng.choice(np.array([rng.integers(0, 65), 200, 1024, 1025, 5000, 64, 65, 0]), n)
        lens = np.where(rng.random(n) < 0.5, rng.integers(0, 65, n), lens)
    elif mix == "lane_then_large":
        lens = np.concatenate([rng.integers(0, 65, n // 2), rng.integers(65, 20000, n - n // 2)])
    elif mix == "random_offsets":
        lens = rng.integers(0, 3000, n)
    else:
        lens = rng.integers(0, 65, n)
    if mix == "random_offsets":
        offs = rng.integers(0, int(lens.sum()), n)
    else:
        offs = np.concatenate([[0], np.cumsum(lens[:-1])]) + rng.integers(0, 9, n).cumsum()
    size = int((offs + lens).max()) + (0 if mix == "lane_at_buffer_end" else 24)
    host = rng.integers(0, 256, size, dtype=np.uint8)
    d = torch.from_numpy(host).to(gpu)
    o = torch.from_numpy(offs.astype(np.int64)).to(gpu)
    ln = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    want = oracle.batch(host, offs, lens.astype(np.int32))
    assert np.array_equal(u32(tk.crc32_batch(d, o, ln)), want)
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    got = u32(tk.crc32_batch(d, o, ln, init_raw=i32(init).to(gpu)))
    assert np.array_equal(got, oracle.batch(host, offs, lens.astype(np.int32), init))
    m = 3000
    got = u32(tk.crc32_batch(d, o[:m].contiguous(), ln[:m].contiguous(), algo="crc32c"))
    assert np.array_equal(got, oracle_c(oracle, host, offs[:m], lens[:m]))


@pytest.mark.parametrize("group_stream", [0, 1])
def test_stream_mode_needs_blocks_longer_than_lanes(gpu, oracle, buf, group_stream):
    """Back-to-back 64-byte blocks are lane blocks (general path). Back-to-back 65-byte blocks are group
    blocks: by default their tiles take the general path and the group phase (round 4; it folds them
    faster than the stream walk's rows of 63 block ends), with tkv_debug_set_stream_groups(1) stream
    mode as before; 300-byte blocks likewise (the small phase), 2000-byte ones stream mode either way.
    All bit-exact."""
    host, d = buf
    lib = tk.load_library()
    prev = lib.tkv_debug_set_stream_groups(group_stream)
    try:
        for blen, want_mode in ((64, 0), (65, group_stream), (40, 0), (128, group_stream), (300, group_stream),
                                (2000, 1)):
            n = 50_000 if blen < 1000 else 20_000
            offs = 7 + np.arange(n, dtype=np.int64) * blen
            lens = np.full(n, blen, np.int32)
            got = u32(tk.crc32_batch(d, torch.from_numpy(offs).to(gpu), torch.from_numpy(lens).to(gpu)))
            assert mode() == want_mode, blen
            assert np.array_equal(got, oracle.batch(host, offs, lens)), blen
    finally:
        lib.tkv_debug_set_stream_groups(prev)


def test_lane_blocks_then_stream_batch_same_scratch(gpu, oracle, buf):
    """A lane-only batch, a stream-mode batch and a mixed general batch one after the other on one
    stream: the lane count of one batch never leaks into the next."""
    host, d = buf
    rng = np.random.default_rng(77)
    batches = [wal_payloads(rng, 5000, WAL_SIZES, 0),
               (np.arange(3000, dtype=np.int64) * 1000, np.full(3000, 1000, np.int32)),
               (np.arange(4000, dtype=np.int64) * 300, rng.integers(0, 300, 4000).astype(np.int32)),
               wal_payloads(rng, 3, (36,), 5)]
    for offs, lens in batches * 2:
        got = u32(tk.crc32_batch(d, torch.from_numpy(offs).to(gpu), torch.from_numpy(lens).to(gpu)))
        assert np.array_equal(got, oracle.batch(host, offs, lens))


@pytest.mark.parametrize("shape", ["wal_payloads", "mixed_gaps", "back_to_back_128", "back_to_back_128_stream",
                                   "back_to_back_300"])
@pytest.mark.parametrize("tiles", [129, 1025])
def test_irregular_more_than_1024_tiles(gpu, oracle, shape, tiles):
    """Batches of more than 128 prepass tiles of 4096 blocks take the one-workgroup tile-sum scan and
    the looping scatter (rows_finish), and above 1024 tiles (4 M blocks) also the 512-thread tile scan:
    lane-dense tiles (WAL payloads), tiles mixing lane, small and
    large blocks with random gaps, and 128-byte blocks back to back, which take stream mode through
    rows_scan_tiles' verdict with tkv_debug_set_stream_groups(1), the general path by default;
    per-block initial registers on the mixed batch."""
    rng = np.random.default_rng({"wal_payloads": 1, "mixed_gaps": 2, "back_to_back_128": 3, "back_to_back_128_stream": 3,
                                 "back_to_back_300": 4}[shape])
    n = 4096 * tiles - 4096 + 777
    if shape == "wal_payloads":
        offs, lens = wal_payloads(rng, n, WAL_SIZES, 3)
    elif shape == "mixed_gaps":
        lens = np.where(rng.random(n) < 0.6, rng.integers(0, 65, n), rng.integers(65, 1025, n))
        lens[rng.integers(0, n, 50)] = rng.integers(1025, 9000, 50)
        offs = np.concatenate([[0], np.cumsum(lens[:-1])]) + rng.integers(0, 5, n).cumsum()
    else:
        blen = 300 if shape == "back_to_back_300" else 128
        lens = np.full(n, blen)
        offs = 5 + np.arange(n, dtype=np.int64) * blen
    lens = lens.astype(np.int32)
    size = int((offs + lens).max()) + 16
    host = rng.integers(0, 256, size, dtype=np.uint8)
    d = torch.from_numpy(host).to(gpu)
    o = torch.from_numpy(offs.astype(np.int64)).to(gpu)
    ln = torch.from_numpy(lens).to(gpu)
    lib = tk.load_library()
    prev = lib.tkv_debug_set_stream_groups(1 if shape == "back_to_back_128_stream" else 0)
    prev_one = lib.tkv_debug_set_one_pass(0)  # the general path's prepass at these sizes, not the one-pass kernel
    try:
        assert np.array_equal(u32(tk.crc32_batch(d, o, ln)), oracle.batch(host, offs, lens))
        got_mode = mode()
        assert path() == 3
    finally:
        lib.tkv_debug_set_stream_groups(prev)
        lib.tkv_debug_set_one_pass(prev_one)
    # back-to-back blocks longer than kLaneMax take stream mode at any batch size, through
    # rows_scan_tiles' verdict, unless their tiles' bytes are mostly in blocks of at most 1 KiB (128 and
    # 300 B, by default: the group passes and the small phase)
    assert got_mode == (1 if shape == "back_to_back_128_stream" else 0)
    if shape == "mixed_gaps":
        init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        got = u32(tk.crc32_batch(d, o, ln, init_raw=i32(init).to(gpu)))
        assert np.array_equal(got, oracle.batch(host, offs, lens, init))


def phases():
    """General-path phases of the last irregular batch: 1 lane, 2/4/8 the 4/8/16-lane group passes."""
    return tk.load_library().tkv_debug_irregular_phases(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))


def path():
    """Which path folded the last irregular batch: 0 crc_list_lanes, 1 its packed mode, 2 the general
    path after both, 3 the general path alone (tkv_debug_irregular_path)."""
    return tk.load_library().tkv_debug_irregular_path(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))


@pytest.mark.parametrize("sizes", [(257,), (300,), (512,), tuple(range(257, 513)), (513,), (700, 1000),
                                   tuple(range(513, 1025)), (1024,), tuple(range(257, 1025))])
@pytest.mark.parametrize("base", [0, 5, 8])
def test_irregular_group8_and_small_blocks(gpu, oracle, buf, sizes, base):
    """Irregular blocks of 257-1024 bytes (WAL payloads with mid-size values): the 8-lane group pass
    (257-512 B, 512-byte slots) in tiles at least half of whose blocks are in its class, the listed
    small phase (1 KiB slots) otherwise: every length at every base alignment, gapped, with per-block
    initial registers and CRC-32C."""
    host, d = buf
    rng = np.random.default_rng(sum(sizes) + base)
    n = min(60_000, (host.size - 64) // (max(sizes) + 8))
    offs, lens = wal_payloads(rng, n, sizes, base)
    o, ln = torch.from_numpy(offs).to(gpu), torch.from_numpy(lens).to(gpu)
    got = u32(tk.crc32_batch(d, o, ln))
    assert mode() == 0
    assert phases() == phases_expected(lens)
    if lens.max() <= 512:
        assert phases() == 4  # the 8-lane pass ran
    assert np.array_equal(got, oracle.batch(host, offs, lens))
    init = rng.integers(0, 2**32, offs.size, dtype=np.uint64).astype(np.uint32)
    got = u32(tk.crc32_batch(d, o, ln, init_raw=i32(init).to(gpu)))
    assert np.array_equal(got, oracle.batch(host, offs, lens, init))
    m = 5000
    got = u32(tk.crc32_batch(d, o[:m].contiguous(), ln[:m].contiguous(), algo="crc32c"))
    assert np.array_equal(got, oracle_c(oracle, host, offs[:m], lens[:m]))


def lists():
    """(listed small blocks, of which <= 256 B, of which 257-512 B) of the last irregular batch."""
    out = (ctypes.c_uint32 * 3)()
    assert tk.load_library().tkv_debug_irregular_lists(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream), out) == 0
    return tuple(int(x) for x in out)


@pytest.mark.parametrize("shape", ["sparse", "dense_g8", "dense_lanes", "tiny"])
@pytest.mark.parametrize("base", [0, 5, 8])
def test_irregular_small_lists_by_class(gpu, oracle, buf, shape, base):
    """Small blocks the lane and group passes do not take are listed by class and folded by 4-, 8- or
    16-lane groups (256-, 512- and 1024-byte slots): every length 0-1024 mixed with large blocks (tiles
    with too many rows for the group passes), next to tiles dense in 257-512-byte blocks (the 8-lane
    pass takes those, the rest stay listed) or in lane blocks; the list sizes the prepass publishes,
    the results, per-block initial registers and CRC-32C."""
    host, d = buf
    rng = np.random.default_rng(700 + base + len(shape))
    if shape == "tiny":  # fewer blocks than one step of each walk
        lens = np.array([0, 1, 256, 257, 512, 513, 1024, 5000], np.int64)
    else:
        n = 24_000
        lens = rng.integers(0, 1025, n)
        big = rng.random(n) < 0.3
        lens[big] = rng.integers(4097, 9000, int(big.sum()))
        if shape == "dense_g8":  # the second and fourth tiles: 257-512-byte blocks only, no large ones
            for t in (1, 3):
                lens[t * 4096:(t + 1) * 4096] = rng.integers(257, 513, 4096)
        if shape == "dense_lanes":  # the third tile: mostly lane blocks
            lens[2 * 4096:3 * 4096] = np.where(rng.random(4096) < 0.5, rng.integers(0, 65, 4096), rng.integers(65, 1025, 4096))
        lens[:1025] = np.arange(1025)  # every small length, all in the first tile
        lens[1025:1025 + 200] = rng.integers(5000, 9000, 200)  # keeps the first tile out of the group passes
    gaps = rng.integers(0, 9, lens.size)
    offs = base + np.concatenate([[0], np.cumsum(lens[:-1] + gaps[:-1])])
    assert offs[-1] + lens[-1] <= host.size
    o, ln = torch.from_numpy(offs.astype(np.int64)).to(gpu), torch.from_numpy(lens.astype(np.int32)).to(gpu)
    got = u32(tk.crc32_batch(d, o, ln))
    assert mode() == 0
    assert lists() == lists_expected(lens)
    assert phases() == phases_expected(lens)
    assert np.array_equal(got, oracle.batch(host, offs, lens))
    init = rng.integers(0, 2**32, offs.size, dtype=np.uint64).astype(np.uint32)
    got = u32(tk.crc32_batch(d, o, ln, init_raw=i32(init).to(gpu)))
    assert np.array_equal(got, oracle.batch(host, offs, lens, init))
    got = u32(tk.crc32_batch(d, o, ln, algo="crc32c"))
    assert np.array_equal(got, oracle_c(oracle, host, offs, lens))


@pytest.mark.parametrize("pattern", ["all_1024", "empty_mix", "one_byte_mix", "16_lanes", "2_lanes", "ramp", "one"])
def test_irregular_small_packed_lanes(gpu, oracle, buf, pattern):
    """Listed small blocks of every lane count (ceil(len / 64) = 1..16) in the small-block phase's class
    walks: whole 1 KiB slots, empty blocks, one-byte blocks among 1 KiB ones, blocks of exactly 16
    lanes, 2-lane blocks, ramps of every length, and a single block; each beside large blocks so that
    no group pass takes them, at base offsets 0-7. (Round 4 also built a walk that packed such blocks
    back to back in lane space; this test was written for it, and it measured slower)"""
    host, d = buf
    rng = np.random.default_rng(len(pattern) * 7)
    n = 9000
    # (lane blocks stay under the lane phase's 256 per tile, so they are listed too)
    small = {"all_1024": np.full(n, 1024),
             "empty_mix": np.where(rng.random(n) < 0.1, 0, rng.integers(500, 1025, n)),
             "one_byte_mix": np.tile([1] + [1024] * 9, n // 10), "16_lanes": rng.integers(961, 1025, n),
             "2_lanes": rng.integers(65, 129, n), "ramp": np.arange(n) % 1025,
             "one": np.array([777])}[pattern].astype(np.int64)
    lens = np.empty(small.size * 2, np.int64)
    lens[0::2] = small
    lens[1::2] = 4097 + rng.integers(0, 3000, small.size)  # rows enough to keep every group pass off
    for base in range(8):
        gaps = rng.integers(1, 5, lens.size)  # (gapped: back-to-back pairs could take stream mode)
        offs = base + np.concatenate([[0], np.cumsum(lens[:-1] + gaps[:-1])])
        if offs[-1] + lens[-1] > host.size:
            keep = int(np.searchsorted(offs + lens, host.size, side="right"))
            offs, lens_b = offs[:keep], lens[:keep]
        else:
            lens_b = lens
        o = torch.from_numpy(offs.astype(np.int64)).to(gpu)
        ln = torch.from_numpy(lens_b.astype(np.int32)).to(gpu)
        got = u32(tk.crc32_batch(d, o, ln))
        assert mode() == 0 and phases() == phases_expected(lens_b) == 0, base
        assert lists() == lists_expected(lens_b), base
        want = oracle.batch(host, offs, lens_b)
        bad = np.flatnonzero(got != want)
        assert bad.size == 0, (base, bad[:5], lens_b[bad[:5]])


@pytest.mark.parametrize("sizes", [(65,), (100, 128, 200), tuple(range(65, 257)), (256,)])
@pytest.mark.parametrize("base", [0, 5, 8])
def test_irregular_group_blocks(gpu, oracle, buf, sizes, base):
    """Irregular blocks of 65-256 bytes in dense tiles (WAL records with short values: gapped payloads)
    are folded by the group phase, a 4-lane group per block right-aligned in a 256-byte slot, at every
    base alignment; per-block initial registers and CRC-32C on the same batch."""
    host, d = buf
    rng = np.random.default_rng(len(sizes) * 31 + base)
    offs, lens = wal_payloads(rng, 100_000, sizes, base)
    o, ln = torch.from_numpy(offs).to(gpu), torch.from_numpy(lens).to(gpu)
    got = u32(tk.crc32_batch(d, o, ln))
    assert mode() == 0
    assert np.array_equal(got, oracle.batch(host, offs, lens))
    init = rng.integers(0, 2**32, offs.size, dtype=np.uint64).astype(np.uint32)
    got = u32(tk.crc32_batch(d, o, ln, init_raw=i32(init).to(gpu)))
    assert np.array_equal(got, oracle.batch(host, offs, lens, init))
    m = 2000
    got = u32(tk.crc32_batch(d, o[:m].contiguous(), ln[:m].contiguous(), algo="crc32c"))
    assert np.array_equal(got, oracle_c(oracle, host, offs[:m], lens[:m]))


def test_irregular_lane_group_small_mix(gpu, oracle):
    """Lane (<= 64 B), group (65-256 B), small (257 B - 1 KiB) and large blocks in one batch, dense and
    sparse tiles (a sparse tile lists its group blocks as small blocks; a tile can be dense in lane
    blocks and sparse in group blocks, or the reverse, or too large in bytes for the group phase),
    random gaps and a batch that ends on the tensor's last byte."""
    rng = np.random.default_rng(4242)
    n = 4096 * 6 + 123
    lens = rng.integers(0, 257, n)
    lens[4096 * 2:4096 * 3] = rng.choice([300, 700, 1024, 5000, 100], 4096)  # a sparse tile
    # dense lane blocks beside sparse group blocks, then the other way round
    lens[4096 * 4:4096 * 5] = rng.choice([10, 100, 300, 700, 2000], 4096)
    lens[4096 * 5:4096 * 6] = rng.choice([100, 150, 200, 300, 1500], 4096)
    lens[4096 * 5 + rng.integers(0, 4096, 200)] = 5
    lens[[4096 * 3 + 7, 4096 * 3 + 900]] = [3 << 20, 2 << 20]  # group-dense, but over kGroupTileBytes
    lens[rng.integers(0, n, 40)] = rng.integers(1025, 20000, 40)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])]) + rng.integers(0, 17, n).cumsum()
    size = int((offs + lens).max())
    host = rng.integers(0, 256, size, dtype=np.uint8)
    d = torch.from_numpy(host).to(gpu)
    o = torch.from_numpy(offs.astype(np.int64)).to(gpu)
    ln = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    assert np.array_equal(u32(tk.crc32_batch(d, o, ln)), oracle.batch(host, offs, lens.astype(np.int32)))
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    got = u32(tk.crc32_batch(d, o, ln, init_raw=i32(init).to(gpu)))
    assert np.array_equal(got, oracle.batch(host, offs, lens.astype(np.int32), init))
