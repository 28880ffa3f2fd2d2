"""GPU parity of crc_list_lanes' packed mode: the one-pass kernel folds an irregular
batch of blocks of at most 1 KiB (default initial register, at least 256 K blocks); a wave switches to
the packed mode at its first step with a block over 64 B, where each block gets ceil(len / 64) lanes
packed back to back over 64-block chunks, every lane folds one 64-byte piece, moves it to the block
end and XORs it into the block's LDS accumulator.

The shapes are the reference's WAL payloads with short and mid-size values (record_len = 18 + |k| +
|v|, /root/reference/src/engine/wal.cpp:25, 8 header bytes before each payload, wal.cpp:54-58) and
blocks of any length 0-1024 in any layout (gapped, back to back, out of order, overlapping, ending at
the allocation's last byte). Every block is compared with the oracle (oracle/crc32_oracle.c, the
reference's crc32.cpp:9-22); tkv_debug_irregular_path says which kernel folded the batch, so a batch
with one block over 1 KiB is checked to take the general path, and one of lane blocks only to stay
with crc_list_lanes.
"""
import ctypes

import numpy as np
import pytest

import tinykvpp_amd as tk

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

N = 1_100_003  # >= 256 K blocks (the one-pass kernel's threshold), not a multiple of 64


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def path():
    return tk.load_library().tkv_debug_irregular_path(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))


def phases():
    return tk.load_library().tkv_debug_irregular_phases(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))


@pytest.fixture(scope="module")
def buf(gpu):
    rng = np.random.default_rng(1024)
    host = rng.integers(0, 256, (256 << 20) + 4096, dtype=np.uint8)
    return host, torch.from_numpy(host).to(gpu)


def gapped(rng, lens, base, gap_hi=9):
    """Offsets of blocks laid out in order with 0..gap_hi-1 bytes between them."""
    gaps = rng.integers(0, gap_hi, lens.size)
    return (base + np.concatenate([[0], np.cumsum(lens[:-1] + gaps[:-1])])).astype(np.int64)


def oracle_c(oracle, host, offs, lens):
    out = np.zeros(len(offs), np.uint32)
    for i, (o, n) in enumerate(zip(offs, lens)):
        out[i] = oracle.update_c(0xFFFFFFFF, host[int(o):int(o) + int(n)].tobytes()) ^ 0xFFFFFFFF
    return out


SHAPES = ["wal_65_256", "wal_100_200", "mix_0_1024", "all_1024", "back_to_back_128", "shuffled", "overlapping",
          "zero_heavy", "lanes_then_pack", "spread_lanes", "late_huge", "early_huge", "mid_huge", "at_allocation_end",
          "at_allocation_start", "page_edges", "crc32c"]


@pytest.mark.parametrize("shape", SHAPES)
def test_pack_one_pass(gpu, oracle, buf, shape):
    host, d = buf
    rng = np.random.default_rng(sum(map(ord, shape)))
    n = N
    want_path = 1
    if shape in ("wal_65_256", "crc32c"):
        lens = rng.integers(65, 257, n)
        offs = 3 + 8 + np.concatenate([[0], np.cumsum(lens[:-1] + 8)])
    elif shape == "wal_100_200":
        lens = rng.integers(100, 201, n)
        offs = 5 + 8 + np.concatenate([[0], np.cumsum(lens[:-1] + 8)])
    elif shape in ("mix_0_1024", "late_huge", "early_huge", "mid_huge"):
        lens = rng.integers(0, 1025, n)
        offs = rng.integers(0, host.size - 1024 - 8192, n)  # overlapping, any order
        if shape != "mix_0_1024":
            at = {"late_huge": n - 5, "early_huge": 3, "mid_huge": n // 2}[shape]
            lens[at] = {"late_huge": 1025, "early_huge": 1025, "mid_huge": 5000}[shape]
            want_path = 2
    elif shape == "all_1024":  # 16 lanes per block: 16 substeps per chunk
        lens = np.full(n, 1024)
        offs = rng.integers(0, host.size - 1024, n)
    elif shape == "back_to_back_128":
        lens = np.full(n, 128)
        offs = 7 + np.arange(n, dtype=np.int64) * 128
        offs %= host.size - 8192
    elif shape == "shuffled":
        lens = rng.integers(26, 400, n)
        offs = gapped(rng, lens, 1)
        p = rng.permutation(n)
        offs, lens = offs[p], lens[p]
    elif shape == "overlapping":
        lens = rng.integers(0, 1025, n)
        offs = np.sort(rng.integers(0, 40 << 20, n))
    elif shape == "zero_heavy":  # chunks with no piece at all
        lens = np.where(rng.random(n) < 0.97, 0, rng.integers(0, 1025, n))
        lens[: 64 * 50] = 0
        offs = gapped(rng, lens, 2)
    elif shape == "lanes_then_pack":  # crc_list_lanes folds its first waves' steps, then hands on
        lens = np.concatenate([rng.integers(0, 65, n // 2), rng.integers(0, 700, n - n // 2)])
        offs = gapped(rng, lens, 6)
    elif shape == "spread_lanes":  # lane blocks whose first steps fit no window: the packed mode, one lane each
        lens = rng.integers(0, 65, n)
        offs = rng.integers(0, host.size - 64, n)
    elif shape == "at_allocation_end":  # every block ends on a 1 KiB slot's last byte, the last on the tensor's
        lens = rng.integers(0, 1025, n)
        offs = (host.size - 1024 * 64 + 1024 * (np.arange(n) % 64) + (1024 - lens)).astype(np.int64)
    elif shape == "page_edges":  # blocks starting 0-31 bytes into a 4 KiB page (the 16-byte-granule loads)
        lens = rng.integers(0, 1025, n)
        offs = 4096 * rng.integers(0, (host.size >> 12) - 1, n) + rng.integers(0, 32, n)
    elif shape == "at_allocation_start":  # every block starts a 1 KiB slot, the first at the tensor's first byte
        lens = rng.integers(0, 1025, n)
        offs = (1024 * (np.arange(n) % 64)).astype(np.int64)
    offs = np.asarray(offs, np.int64)
    lens = np.asarray(lens, np.int32)
    assert int((offs + lens).max()) <= host.size
    o, ln = torch.from_numpy(offs).to(gpu), torch.from_numpy(lens).to(gpu)
    if shape == "crc32c":
        got = u32(tk.crc32_batch(d, o, ln, algo="crc32c"))
        assert path() == 1
        sample = rng.choice(n, 20_000, replace=False)
        assert np.array_equal(got[sample], oracle_c(oracle, host, offs[sample], lens[sample]))
        return
    got = u32(tk.crc32_batch(d, o, ln))
    assert path() == want_path, shape
    if want_path == 1:
        assert phases() == 0
    want = oracle.batch(host, offs, lens)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (shape, bad.size, bad[:5], lens[bad[:5]])
    if shape == "at_allocation_end":  # the same blocks in a copy whose last byte is the allocation's last
        cut = host.size - 1024 * 64
        tail = d[cut:].clone()
        got = u32(tk.crc32_batch(tail, torch.from_numpy(offs - cut).to(gpu), ln))
        assert path() == 1
        assert np.array_equal(got, want)
    if shape == "at_allocation_start":  # a fresh copy of the first 64 KiB: no load may reach in front of it
        head = torch.empty(64 << 10, dtype=torch.uint8, device=gpu)
        head.copy_(d[:64 << 10])
        got = u32(tk.crc32_batch(head, o, ln))
        assert path() == 1
        assert np.array_equal(got, want)


def test_pack_paths_one_after_another(gpu, oracle, buf):
    """Batches on one stream whose verdicts alternate: lane blocks only (crc_list_lanes), blocks up to
    1 KiB (the packed mode), one block over 1 KiB (the general path), and again; a stale flag of one call
    never steers the next (each call's flags carry its own sequence number)."""
    host, d = buf
    rng = np.random.default_rng(5)
    lane_lens = rng.integers(26, 60, N)
    lane_offs = 11 + np.concatenate([[0], np.cumsum(lane_lens[:-1] + 8)])
    pack_lens = rng.integers(0, 1025, N)
    pack_offs = rng.integers(0, host.size - 1024, N)
    big_lens = pack_lens.copy()
    big_lens[N // 3] = 3000
    cases = [(lane_offs, lane_lens, 0), (pack_offs, pack_lens, 1), (pack_offs, big_lens, 2)]
    for offs, lens, want_path in cases + cases[::-1]:
        offs, lens = np.asarray(offs, np.int64), np.asarray(lens, np.int32)
        got = u32(tk.crc32_batch(d, torch.from_numpy(offs).to(gpu), torch.from_numpy(lens).to(gpu)))
        assert path() == want_path
        assert np.array_equal(got, oracle.batch(host, offs, lens)), want_path


def test_pack_not_with_per_block_registers(gpu, oracle, buf):
    """Per-block initial registers keep the general path (the one-pass kernel folds from the default
    register only): same results as the oracle, path 3."""
    host, d = buf
    rng = np.random.default_rng(9)
    lens = rng.integers(65, 1025, N).astype(np.int32)
    offs = rng.integers(0, host.size - 1024, N).astype(np.int64)
    init = rng.integers(0, 2**32, N, dtype=np.uint64).astype(np.uint32)
    got = u32(tk.crc32_batch(d, torch.from_numpy(offs).to(gpu), torch.from_numpy(lens).to(gpu),
                             init_raw=torch.from_numpy(init.view(np.int32)).to(gpu)))
    assert path() == 3
    assert np.array_equal(got, oracle.batch(host, offs, lens, init))


@pytest.mark.parametrize("n,want_path", [(262_144, 1), (262_143, 3)])
def test_pack_threshold(gpu, oracle, buf, n, want_path):
    """The one-pass kernel takes batches of at least 256 K blocks (kListMinBlocks); one block fewer
    takes the general path alone. Same results either way; tkv_debug_set_one_pass(0) sends the larger
    batch to the general path too."""
    host, d = buf
    rng = np.random.default_rng(n)
    lens = rng.integers(65, 257, n).astype(np.int32)
    offs = (3 + 8 + np.concatenate([[0], np.cumsum(lens[:-1] + 8)])).astype(np.int64)
    o, ln = torch.from_numpy(offs).to(gpu), torch.from_numpy(lens).to(gpu)
    want = oracle.batch(host, offs, lens)
    assert np.array_equal(u32(tk.crc32_batch(d, o, ln)), want)
    assert path() == want_path
    lib = tk.load_library()
    prev = lib.tkv_debug_set_one_pass(0)
    try:
        assert np.array_equal(u32(tk.crc32_batch(d, o, ln)), want)
        assert path() == 3
    finally:
        lib.tkv_debug_set_one_pass(prev)


@pytest.mark.parametrize("mix", ["lanes", "packed"])
def test_one_pass_offsets_past_4_gib(gpu, oracle, mix):
    """Block offsets on both sides of 4 GiB (u64 offsets; 32-bit arithmetic only relative to a block):
    gapped WAL payloads of 26-59 B (lane mode) or 0-1024 B (packed mode) running across byte 2^32 of a
    4.5 GiB device buffer. Only the bytes the blocks touch are written; the oracle sees the same bytes
    at offsets relative to that window."""
    rng = np.random.default_rng(4 << 30 if mix == "lanes" else 5 << 30)
    n = 600_000 if mix == "lanes" else 300_000
    lens = (rng.integers(26, 60, n) if mix == "lanes" else rng.integers(0, 1025, n)).astype(np.int64)
    rel = np.concatenate([[0], np.cumsum(lens[:-1] + 8)])
    span = int(rel[-1] + lens[-1])
    lo = (1 << 32) - span // 2 - 8  # the window straddles 2^32
    host = rng.integers(0, 256, span + 64, dtype=np.uint8)
    d = torch.empty((9 << 29), dtype=torch.uint8, device=gpu)  # 4.5 GiB
    d[lo:lo + host.size] = torch.from_numpy(host).to(gpu)
    offs = (lo + rel).astype(np.int64)
    got = u32(tk.crc32_batch(d, torch.from_numpy(offs).to(gpu), torch.from_numpy(lens.astype(np.int32)).to(gpu)))
    assert path() == (0 if mix == "lanes" else 1)
    want = oracle.batch(host, rel, lens.astype(np.int32))
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (mix, bad.size, bad[:5], offs[bad[:5]])
    del d
