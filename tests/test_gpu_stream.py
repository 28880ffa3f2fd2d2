"""Irregular batches whose blocks lie back to back (each longer than kLaneMax = 64 bytes) take the byte-stream row
walk: the prepass chooses it on the device, the row kernel walks full 4 KiB rows of
the stream and records a (Y, Q) pair at every block end and a register per wave, and the general row
kernel's launch (which has no rows to walk then) turns those into block CRCs. Every case is compared block by block with the oracle (crc32.cpp:9-16 restated),
and the path actually taken is read back with tkv_debug_irregular_mode."""
import ctypes

import numpy as np
import pytest
import torch

import tinykvpp_amd as tk
from conftest import stream_expected

pytestmark = pytest.mark.gpu


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def mode():
    return tk.load_library().tkv_debug_irregular_mode(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))


def run(gpu, oracle, lens, start=0, init=False, algo="crc32", seed=0):
    rng = np.random.default_rng(seed)
    lens = np.asarray(lens, np.int64)
    offs = (np.concatenate([[0], np.cumsum(lens[:-1])]) + start).astype(np.int64)
    size = int(offs[-1] + lens[-1]) + 64
    host = rng.integers(0, 256, size, dtype=np.uint8)
    d = torch.from_numpy(host).to(gpu)
    o = torch.from_numpy(offs).to(gpu)
    ln = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    ini = None
    if init:
        ini = rng.integers(0, 2**32, lens.size, dtype=np.uint64).astype(np.uint32)
    got = u32(tk.crc32_batch(d, o, ln, init_raw=None if ini is None else torch.from_numpy(ini.view(np.int32)).to(gpu),
                             algo=algo))
    m = mode()
    if algo == "crc32":
        want = oracle.batch(host, offs, lens, ini)
    else:
        want = np.array([oracle.update_c(0xFFFFFFFF if ini is None else int(ini[i]),
                                         host[offs[i]:offs[i] + lens[i]].tobytes()) ^ 0xFFFFFFFF
                         for i in range(lens.size)], np.uint32)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, f"{bad.size} blocks differ, first {bad[:5]} (mode {m})"
    return m


@pytest.mark.parametrize("start", [0, 1, 7, 15, 16, 4095, 4096 + 9])
def test_stream_alignments(gpu, oracle, start):
    rng = np.random.default_rng(start)
    lens = rng.integers(65, 20000, 3000)
    assert run(gpu, oracle, lens, start=start, seed=start) == 1


def shape_lens(case):
    rng = np.random.default_rng(sum(map(ord, case)))
    if case == "exact64":  # a block end in 64 of every 65 lane segments (64-byte blocks are lane blocks)
        lens = np.full(20000, 65)
    elif case == "seg_ends":  # ends on 64-byte segment boundaries, some at r = 64, some mid-dword
        lens = rng.choice([129, 128, 192, 65, 67, 127], 20000)
    elif case == "row_ends":  # ends on 4 KiB row boundaries
        lens = np.tile([4096, 8192, 4031, 65, 4096 * 3], 500)
    elif case == "one_block":
        lens = np.array([(5 << 20) + 3])
    elif case == "two_blocks":
        lens = np.array([65, 100])
    elif case == "mixed_huge":  # Zipf-like: 256 B to 1 MiB (cfg4's classes)
        lens = np.maximum(256, (256 * 2 ** rng.integers(0, 13, 4000)) - rng.integers(0, 128, 4000))
    elif case == "span_waves":  # blocks that span many waves' row ranges, between small ones
        lens = np.concatenate([rng.integers(65, 5000, 3000), [(40 << 20) + 17], rng.integers(65, 300, 500),
                               [(24 << 20) + 4096], rng.integers(65, 5000, 3000)])
    else:  # many small blocks: several ends per row in consecutive lanes
        lens = rng.integers(65, 200, 200000)
    return lens


SHAPES = ["exact64", "seg_ends", "row_ends", "one_block", "two_blocks", "mixed_huge", "many_small", "span_waves"]


@pytest.mark.parametrize("case", SHAPES)
def test_stream_shapes(gpu, oracle, stream_groups, case):
    """Every shape through the byte-stream walk (with tkv_debug_set_stream_groups(1), so the shapes
    dense in 65-256-byte blocks, whose rows hold 16-64 block ends, take it too)."""
    assert run(gpu, oracle, shape_lens(case), start=5, seed=1) == 1


@pytest.mark.parametrize("case", SHAPES)
def test_stream_shapes_default_policy(gpu, oracle, case):
    """The same shapes with the default policy: back-to-back batches dense in 65-256-byte blocks take
    the general path (their group phase, round 4), the others stream mode; bit-exact either way."""
    lens = shape_lens(case)
    offs = 5 + np.concatenate([[0], np.cumsum(lens[:-1])])
    assert run(gpu, oracle, lens, start=5, seed=1) == stream_expected(offs, lens)
    if case in ("exact64", "seg_ends", "many_small"):
        assert stream_expected(offs, lens) == 0


def test_stream_init_and_crc32c(gpu, oracle):
    rng = np.random.default_rng(11)
    lens = rng.integers(65, 9000, 5000)
    assert run(gpu, oracle, lens, start=3, init=True, seed=2) == 1
    assert run(gpu, oracle, lens, start=3, algo="crc32c", seed=3) == 1
    assert run(gpu, oracle, lens, start=3, init=True, algo="crc32c", seed=4) == 1


def test_general_path_when_not_back_to_back(gpu, oracle):
    """A short block, or a gap between blocks, keeps the general row walk (and stays exact)."""
    rng = np.random.default_rng(12)
    lens = rng.integers(65, 9000, 3000)
    lens[1234] = 63
    assert run(gpu, oracle, lens, seed=5) == 0
    lens = rng.integers(65, 9000, 3000)
    offs = (np.concatenate([[0], np.cumsum(lens[:-1])])).astype(np.int64)
    offs[2000:] += 1  # one byte gap
    host = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
    got = u32(tk.crc32_batch(torch.from_numpy(host).to(gpu), torch.from_numpy(offs).to(gpu),
                             torch.from_numpy(lens.astype(np.int32)).to(gpu)))
    assert mode() == 0
    assert np.array_equal(got, oracle.batch(host, offs, lens))


def test_stream_then_general_on_same_scratch(gpu, oracle):
    """The stream and general paths share the stream's prepass scratch: alternate them."""
    rng = np.random.default_rng(13)
    for k in range(3):
        lens = rng.integers(65, 30000, 2000)
        assert run(gpu, oracle, lens, start=k, seed=20 + k) == 1
        lens[7] = 10
        assert run(gpu, oracle, lens, start=k, seed=30 + k) == 0


@pytest.mark.parametrize("nblocks", [1, 2, 300])
def test_stream_row0_before_a_misaligned_base(gpu, oracle, nblocks):
    """A base pointer that is not 16-byte aligned, with the stream starting in its first bytes: row 0
    (the stream start rounded down to 16 bytes) then starts before the base pointer. Its offset from
    base wraps as a u64; the row count must still come out right (it read 0 rows, and every CRC was
    wrong, for base shifts 1-7 with the stream at offset 8, before the fix)."""
    rng = np.random.default_rng(nblocks)
    lens = rng.integers(65, 9000, nblocks)
    for shift in range(16):
        for first in (0, 3, 8, 15):
            offs = (first + np.concatenate([[0], np.cumsum(lens[:-1])])).astype(np.int64)
            size = int(offs[-1] + lens[-1]) + 64
            host = rng.integers(0, 256, size, dtype=np.uint8)
            d = torch.zeros(size + shift, dtype=torch.uint8, device=gpu)
            d[shift:] = torch.from_numpy(host).to(gpu)
            got = u32(tk.crc32_batch(d[shift:], torch.from_numpy(offs).to(gpu),
                                     torch.from_numpy(lens.astype(np.int32)).to(gpu)))
            assert mode() == 1
            want = oracle.batch(host, offs, lens)
            assert np.array_equal(got, want), (shift, first)
