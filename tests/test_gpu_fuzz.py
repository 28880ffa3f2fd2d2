"""Seeded randomized parity sweep of every device entry point against the oracle (TEST
INFRASTRUCTURE: oracle/liboracle.so is the checker). Each case draws a batch shape the targeted tests
cover one at a time, mixed: lengths 0-3, around the 64-byte lane segment, the 1 KiB small-block
bound and the 4 KiB row, up to 300 KiB; base misalignment 0-4105; back-to-back layouts (stream mode
when every block is >= 64 bytes), overlapping and gapped layouts (general walk), optional per-block
initial registers, both polynomials. The reference's semantics per block: crc32.cpp:9-16 from the
given raw register, finalize() = crc32.cpp:19."""
import ctypes

import numpy as np
import pytest
import torch

import tinykvpp_amd as tk
from conftest import phases_expected, stream_expected

pytestmark = pytest.mark.gpu

# TKV_FUZZ_OFFSET shifts every case's seed, so the same sweep can explore other cases (the default,
# 0, is the committed set).
import os  # noqa: E402
OFFSET = int(os.environ.get("TKV_FUZZ_OFFSET", "0"))

ALGOS = ("crc32", "crc32c")


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def draw_lengths(rng, n):
    """A mixture over the decomposition's boundaries (segment 64 B, small 1 KiB, row 4 KiB)."""
    kind = rng.integers(0, 6, n)
    edges = np.array([0, 1, 2, 3, 63, 64, 65, 1023, 1024, 1025, 4095, 4096, 4097, 8192, 65536])
    lens = np.where(kind == 0, rng.choice(edges, n),
           np.where(kind == 1, rng.integers(0, 64, n),
           np.where(kind == 2, rng.integers(64, 1025, n),
           np.where(kind == 3, rng.integers(1025, 9000, n),
           np.where(kind == 4, rng.integers(9000, 70000, n), rng.integers(70000, 300000, n))))))
    # keep the case's payload bounded so the oracle finishes quickly
    while lens.sum() > (24 << 20):
        lens = lens // 2
    return lens.astype(np.int64)


def oracle_batch(oracle, algo, host, offs, lens, init):
    if algo == "crc32":
        return oracle.batch(host, offs, lens, init)
    out = np.zeros(offs.size, np.uint32)
    for i, (o, n) in enumerate(zip(offs.tolist(), lens.tolist())):
        raw = 0xFFFFFFFF if init is None else int(init[i])
        out[i] = oracle.update_c(raw, host[o:o + n].tobytes()) ^ 0xFFFFFFFF
    return out


def on_device(host, gpu, shift):
    """host bytes on the GPU at `shift` bytes past a 256-byte aligned allocation (the batch APIs take
    any base pointer; stream mode's row 0 may then start before it)."""
    d = torch.zeros(host.size + shift, dtype=torch.uint8, device=gpu)
    d[shift:] = torch.from_numpy(host).to(gpu)
    return d[shift:]


def irregular_mode():
    return tk.load_library().tkv_debug_irregular_mode(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))


def irregular_phases():
    return tk.load_library().tkv_debug_irregular_phases(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))


@pytest.mark.parametrize("seed", range(96))
def test_irregular_random(gpu, oracle, seed):
    rng = np.random.default_rng(1000 + seed + OFFSET)
    algo = ALGOS[seed % 2]
    n = int(rng.choice([1, 2, 3, 17, 300, 2000, 9000]))
    lens = draw_lengths(rng, n)
    layout = ("back_to_back", "back_to_back_min64", "gapped", "overlapping")[seed // 2 % 4]
    if layout == "back_to_back_min64":
        lens = np.maximum(lens, 65)
    start = int(rng.integers(0, 4106))
    if layout.startswith("back_to_back"):
        offs = start + np.concatenate([[0], np.cumsum(lens)[:-1]])
    elif layout == "gapped":
        offs = start + np.concatenate([[0], np.cumsum(lens + rng.integers(0, 40, n))[:-1]])
    else:
        offs = rng.integers(0, max(1, int(lens.sum()) // 2 + 1), n) + start
    size = int((offs + lens).max()) + 64
    host = rng.integers(0, 256, size, dtype=np.uint8)
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) if rng.random() < 0.5 else None
    shift = int(rng.integers(0, 16)) if seed % 3 else 0
    d = on_device(host, gpu, shift)
    o = torch.from_numpy(offs.astype(np.int64)).to(gpu)
    ln = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    ini = None if init is None else torch.from_numpy(init.view(np.int32)).to(gpu)
    got = u32(tk.crc32_batch(d, o, ln, init_raw=ini, algo=algo))
    want = oracle_batch(oracle, algo, host, offs, lens, init)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (f"{layout} n={n} start={start} shift={shift} algo={algo} mode={irregular_mode()}: "
                           f"{bad.size} blocks differ, first {bad[:5]} (lens {lens[bad[:5]]})")
    if layout == "back_to_back_min64" and n > 1:
        assert irregular_mode() == stream_expected(offs, lens), "the prepass's stream verdict"


@pytest.mark.parametrize("seed", range(48))
def test_irregular_dense_small_random(gpu, oracle, seed):
    """Batches dense in blocks of at most 256 bytes (the lane and group phases): lane
    and group shares around the prepass's per-tile thresholds (256 and 3072 of 4096 blocks), a few
    large blocks that may push a tile over the group phase's row bound, gapped, back-to-back and
    overlapping layouts, random base shifts, initial registers and algorithms."""
    rng = np.random.default_rng(5000 + seed + OFFSET)
    algo = ALGOS[seed % 2]
    n = int(rng.choice([4096, 5000, 9000, 20000, 4096 * 3 + 17]))
    p_lane = float(rng.choice([0.0, 0.05, 0.0625, 0.3, 0.9]))
    p_group = float(rng.choice([0.0, 0.2, 0.3, 0.74, 0.76, 0.9]))
    # the rest: 257-512 B (8-lane pass or listed), 513-1024 B (listed) and 1025-3000 B, in shares around
    # the 8-lane pass's tile threshold (3968 of 4096)
    mid = rng.choice([(0.0, 0.0), (0.25, 0.0), (0.3, 0.5), (0.0, 0.55), (0.45, 0.45), (0.96, 0.0), (0.995, 0.0)])
    u = rng.random(n)
    v = rng.random(n)
    rest = np.where(v < mid[0], rng.integers(257, 513, n),
           np.where(v < mid[0] + mid[1], rng.integers(513, 1025, n), rng.integers(1025, 3000, n)))
    lens = np.where(u < p_lane, rng.integers(0, 65, n),
           np.where(u < p_lane + p_group, rng.integers(65, 257, n), rest))
    nbig = int(rng.choice([0, 1, 3]))
    lens[rng.integers(0, n, nbig)] = rng.integers(1 << 20, 6 << 20, nbig)
    layout = ("gapped", "back_to_back", "overlapping")[seed % 3]
    start = int(rng.integers(0, 300))
    if layout == "back_to_back":
        offs = start + np.concatenate([[0], np.cumsum(lens)[:-1]])
    elif layout == "gapped":
        offs = start + np.concatenate([[0], np.cumsum(lens + rng.integers(0, 20, n))[:-1]])
    else:
        offs = rng.integers(0, max(1, int(lens.sum()) // 2 + 1), n) + start
    host = rng.integers(0, 256, int((offs + lens).max()) + 64, dtype=np.uint8)
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) if seed % 4 < 2 else None
    shift = int(rng.integers(0, 16))
    d = on_device(host, gpu, shift)
    ini = None if init is None else torch.from_numpy(init.view(np.int32)).to(gpu)
    got = u32(tk.crc32_batch(d, torch.from_numpy(offs.astype(np.int64)).to(gpu),
                             torch.from_numpy(lens.astype(np.int32)).to(gpu), init_raw=ini, algo=algo))
    want = oracle_batch(oracle, algo, host, offs, lens, init)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (f"{layout} n={n} lane={p_lane} group={p_group} mid={mid} big={nbig} shift={shift} "
                           f"algo={algo} mode={irregular_mode()}: {bad.size} blocks differ, first {bad[:5]} "
                           f"(lens {lens[bad[:5]]})")
    if irregular_mode() == 0:
        assert irregular_phases() == phases_expected(lens)


@pytest.mark.parametrize("seed", range(64))
def test_uniform_random(gpu, oracle, seed):
    rng = np.random.default_rng(2000 + seed + OFFSET)
    algo = ALGOS[seed % 2]
    length = int(rng.choice([0, 1, 3, 16, 48, 64, 128, 256, 512, 1000, 1024, 1040, 2048, 3008, 4080, 4096, 4097,
                             8192, 12288, 65536, int(rng.integers(0, 70000)), 16 * int(rng.integers(1, 256))]))
    stride = length + int(rng.choice([0, 0, 0, 0, 1, 16, 4096, int(rng.integers(0, 5000))]))
    stride = max(stride, 1)
    n = int(rng.choice([1, 5, 4095, 4096, 5000, 20000]))
    while n * stride > (48 << 20) and n > 1:
        n //= 2
    offset = int(rng.choice([0, 0, 16, int(rng.integers(0, 4106))]))
    size = offset + (n - 1) * stride + length + 64
    host = rng.integers(0, 256, size, dtype=np.uint8)
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) if rng.random() < 0.4 else None
    shift = int(rng.integers(0, 16)) if seed % 3 else 0
    d = on_device(host, gpu, shift)
    ini = None if init is None else torch.from_numpy(init.view(np.int32)).to(gpu)
    got = u32(tk.crc32_batch_uniform(d, length, n, stride=stride, init_raw=ini, offset=offset, algo=algo))
    offs = offset + np.arange(n, dtype=np.int64) * stride
    want = oracle_batch(oracle, algo, host, offs, np.full(n, length, np.int64), init)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, f"len={length} stride={stride} n={n} offset={offset} shift={shift} algo={algo}: {bad[:5]}"


@pytest.mark.parametrize("seed", range(16))
def test_update_chain_random(gpu, oracle, seed):
    """crc32::update chained over random pieces (host spans and device tensors) equals one pass."""
    rng = np.random.default_rng(3000 + seed + OFFSET)
    algo = ALGOS[seed % 2]
    pieces = [rng.integers(0, 256, int(rng.choice([0, 1, 5, 36, 700, 4096, 20000, 300000])), dtype=np.uint8)
              for _ in range(int(rng.integers(1, 12)))]
    c = tk.crc32() if algo == "crc32" else tk.crc32c()
    raw = 0xFFFFFFFF
    for i, p in enumerate(pieces):
        c.update(on_device(p, gpu, int(rng.integers(0, 16))) if i % 2 else p.tobytes())
        raw = oracle.update(raw, p.tobytes()) if algo == "crc32" else oracle.update_c(raw, p.tobytes())
    assert c.finalize() == raw ^ 0xFFFFFFFF


@pytest.mark.parametrize("seed", range(96))
def test_wal_verify_random(gpu, oracle, seed):
    """Device WAL recovery verify (host-image and device-image paths) on random WAL images against
    the sequential decode of wal.cpp:63-130 (test_gpu_wal_device.sequential_decode): random record
    counts and value sizes, values holding fake headers, torn tails, an unaligned device image, and
    one random corruption: a payload bit, the stored CRC, a lying record_len, a key/value length that
    overruns the record under a valid CRC (caught after the CRC, wal.cpp:118-121), or any byte."""
    from test_gpu_wal_device import both, make_wal, sequential_decode
    rng = np.random.default_rng(4000 + seed + OFFSET)
    n_rec = int(rng.choice([1, 2, 7, 300, 5000, 20000, 120000]))
    vmax = int(rng.choice([64, 600, 5000, 16000])) if n_rec < 100000 else 600
    img, offs, size = make_wal(rng, n_rec, vmax=vmax, fake_headers=float(rng.choice([0.0, 0.0, 0.3])))
    kind = ("none", "payload", "crc", "record_len", "kv_overflow", "any")[seed % 6]
    r = int(rng.integers(0, n_rec))
    o = int(offs[r])
    if kind == "payload":
        img[o + 8 + int(rng.integers(0, int(size[r]) - 8))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    elif kind == "crc":
        img[o + 4 + int(rng.integers(0, 4))] ^= np.uint8(0x10)
    elif kind == "record_len":
        delta = int(rng.choice([-9, -1, 1, 5, 4096, 1 << 20]))
        img[o:o + 4] = np.frombuffer(((int(size[r]) - 8 + delta) & 0xFFFFFFFF).to_bytes(4, "little"), np.uint8)
    elif kind == "kv_overflow":
        img[o + 22:o + 26] = np.frombuffer((int(size[r])).to_bytes(4, "little"), np.uint8)  # vlen > what fits
        lib = tk.load_library()
        one_off = np.array([o], np.uint64)
        one_len = np.array([int(size[r])], np.uint32)
        tk.check(lib.tkv_wal_stamp(ctypes.c_void_p(img.ctypes.data), ctypes.c_void_p(one_off.ctypes.data),
                                   ctypes.c_void_p(one_len.ctypes.data), 1))  # a valid CRC over the bad lengths
    elif kind == "any":
        img[int(rng.integers(0, img.size))] ^= np.uint8(int(rng.integers(1, 256)))
    n = img.size if rng.random() < 0.6 else int(rng.integers(0, img.size + 1))  # torn tail
    want = sequential_decode(oracle, img, n)
    if kind == "kv_overflow" and o + int(size[r]) <= n:
        assert want[0] == "corrupted" and want[2] <= o
    got = both(img, n, shift=int(rng.integers(0, 16)))
    assert got == (want, want), f"kind={kind} record={r} n_rec={n_rec} vmax={vmax} n={n}"
    if seed % 3 == 0:  # the host image in pinned memory at any alignment (read in place)
        pshift = int(rng.integers(0, 16))
        pin = torch.empty(n + pshift, dtype=torch.uint8, pin_memory=True)
        pin.numpy()[pshift:] = img[:n]
        assert tk.wal.verify(pin.numpy()[pshift:]) == want, f"pinned shift {pshift}"


@pytest.mark.parametrize("seed", range(48))
def test_host_batch_random(gpu, oracle, seed):
    """tkv_crc32[c]_batch_host[_multi] over pageable host memory (the staged pipeline: dense runs,
    gathers, blocks cut across devices) and pinned host memory (read in place) at any alignment,
    random layouts and initial registers, against the oracle."""
    rng = np.random.default_rng(5000 + seed + OFFSET)
    algo = ALGOS[seed % 2]
    n = int(rng.choice([1, 3, 40, 256, 257, 3000]))
    lens = draw_lengths(rng, n)
    if seed % 5 == 0:  # a few blocks of 1-3 MiB (cut between devices by the multi-device split)
        lens[rng.integers(0, n, 2)] = rng.integers(1 << 20, 3 << 20, 2)
    layout = ("back_to_back", "gapped", "overlapping")[seed % 3]
    if layout == "back_to_back":
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    elif layout == "gapped":
        offs = np.concatenate([[0], np.cumsum(lens + rng.integers(0, 40, n))[:-1]])
    else:
        offs = rng.integers(0, max(1, int(lens.sum()) // 2 + 1), n)
    shift = int(rng.integers(0, 16))
    size = int((offs + lens).max()) + 64
    raw = rng.integers(0, 256, size + shift, dtype=np.uint8)
    pinned = seed % 2 == 1
    if pinned:  # a pinned source: the kernels read it in place over PCIe (mapped_batch)
        pin = torch.empty(size + shift, dtype=torch.uint8, pin_memory=True)
        pin.numpy()[:] = raw
        raw = pin.numpy()
    host = raw[shift:]  # a source at any alignment
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) if rng.random() < 0.4 else None
    devices = (None, [0], [0, 0], [0, 0, 0, 0])[seed % 4]
    got = tk.crc32_batch_host(host, offs.astype(np.uint64), lens.astype(np.uint32), init_raw=init,
                              devices=devices, algo=algo)
    want = oracle_batch(oracle, algo, host, offs.astype(np.int64), lens, init)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, f"{layout} n={n} shift={shift} pinned={pinned} devices={devices} algo={algo}: {bad[:5]}"


@pytest.mark.parametrize("seed", range(24))
def test_sst_random(gpu, oracle, seed):
    """SSTable data-block stamping (format: include/tkv_crc32.h; parity unpinned, checked against
    the oracle's literal restatement): random files at any alignment, host stamp against the oracle,
    device stamp (block_crcs_device, store) against the host stamp, verify of a random corruption."""
    from test_gpu_formats import make_file
    from tinykvpp_amd import sst
    rng = np.random.default_rng(6000 + seed + OFFSET)
    f, offs, sizes = make_file(rng, int(rng.choice([1, 2, 30, 400])))
    shift = int(rng.integers(0, 16))
    buf = np.zeros(f.size + shift, np.uint8)
    host = buf[shift:]
    host[:] = f
    sst.stamp_blocks(host, offs, sizes)
    for o, s in zip(offs.tolist(), sizes.tolist()):
        img = host[o:o + s].tobytes()
        assert int.from_bytes(img[17:21], "little") == oracle.sst_stamp(img)
    assert sst.verify_blocks(host, offs, sizes) == ("ok", 0, offs.size)
    dshift = int(rng.integers(0, 16))
    garbage = f.copy()
    garbage[offs.astype(np.int64)[:, None] + np.arange(17, 21)] = rng.integers(0, 256, (offs.size, 4), dtype=np.uint8)
    d = on_device(garbage, gpu, dshift)
    o = torch.from_numpy(offs.astype(np.int64)).to(gpu)
    sz = torch.from_numpy(sizes.astype(np.int32)).to(gpu)
    sst.block_crcs_device(d, o, sz, store=True)
    assert np.array_equal(d.cpu().numpy(), host), f"device stamp differs (shift {dshift})"
    victim = int(rng.integers(0, offs.size))
    pos = int(offs[victim]) + int(rng.integers(0, int(sizes[victim])))
    host[pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
    assert sst.verify_blocks(host, offs, sizes) == ("corrupted", 1, victim)


@pytest.mark.parametrize("seed", range(16))
def test_wal_stamp_random(gpu, oracle, seed):
    """WAL group-commit stamping (tkv_wal_stamp, wal.cpp:54-58 per record) of random records: the
    CRC over [8, 8 + record_len) of each, stored at offset 4, against the oracle; the stamped batch
    verifies clean."""
    from tinykvpp_amd import wal
    rng = np.random.default_rng(7000 + seed + OFFSET)
    n = int(rng.choice([1, 2, 16, 255, 256, 257, 5000]))
    recs = [wal.encode_unstamped(int(rng.integers(0, 2)), int(rng.integers(0, 2**63)),
                                 rng.bytes(int(rng.integers(0, 64))),
                                 rng.bytes(int(min(rng.zipf(1.5) * 32, 40000))), int(rng.integers(0, 2)))
            for _ in range(n)]
    stamped = wal.stamp(recs)
    for r, s in zip(recs, stamped):
        assert s[:4] == r[:4] and s[8:] == r[8:]
        assert int.from_bytes(s[4:8], "little") == oracle.crc(r[8:])
    image = b"".join(stamped)
    assert wal.verify(image) == ("ok", n, len(image))
    # the same group commit in place in a pinned append buffer at any alignment
    shift = int(rng.integers(0, 16))
    pin = torch.empty(len(image) + shift, dtype=torch.uint8, pin_memory=True)
    buf = pin.numpy()[shift:]
    buf[:] = np.frombuffer(b"".join(recs), np.uint8)
    sizes = np.array([len(r) for r in recs], np.uint32)
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
    tk.check(tk.load_library().tkv_wal_stamp(ctypes.c_void_p(buf.ctypes.data), ctypes.c_void_p(offs.ctypes.data),
                                             ctypes.c_void_p(sizes.ctypes.data), n))
    assert buf.tobytes() == image, f"pinned stamp differs (shift {shift})"


@pytest.mark.parametrize("group_stream", [True, False])
@pytest.mark.parametrize("seed", range(12))
def test_stream_many_blocks_random(gpu, oracle, seed, group_stream):
    """Stream mode over 50 K-200 K back-to-back blocks (several block ends per row and lane segment
    boundary, every wave holding ends), any base alignment and stream start, per-block initial
    registers, both polynomials; with tkv_debug_set_stream_groups(1) every such batch takes the stream
    walk, with the default policy those dense in 65-256-byte blocks take the general path."""
    lib = tk.load_library()
    prev = lib.tkv_debug_set_stream_groups(1 if group_stream else 0)
    try:
        stream_many_case(oracle, gpu, seed, group_stream)
    finally:
        lib.tkv_debug_set_stream_groups(prev)


def stream_many_case(oracle, gpu, seed, group_stream):
    rng = np.random.default_rng(8000 + seed + OFFSET)
    algo = ALGOS[seed % 2]
    n = int(rng.integers(50_000, 200_000))
    lens = rng.integers(65, int(rng.choice([66, 128, 600, 3000])), n).astype(np.int64)
    start = int(rng.integers(0, 64))
    offs = start + np.concatenate([[0], np.cumsum(lens)[:-1]])
    host = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) if seed % 3 == 0 else None
    shift = int(rng.integers(0, 16))
    d = on_device(host, gpu, shift)
    ini = None if init is None else torch.from_numpy(init.view(np.int32)).to(gpu)
    got = u32(tk.crc32_batch(d, torch.from_numpy(offs).to(gpu), torch.from_numpy(lens.astype(np.int32)).to(gpu),
                             init_raw=ini, algo=algo))
    assert irregular_mode() == stream_expected(offs, lens, group_stream)
    want = oracle_batch(oracle, algo, host, offs, lens, init)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, f"n={n} start={start} shift={shift} algo={algo}: {bad.size} differ, first {bad[:5]}"


@pytest.mark.parametrize("seed", range(24))
def test_one_pass_random(gpu, oracle, seed):
    """Batches of at least 256 K blocks with the default register: the one-pass kernel
    (crc_list_lanes and its packed mode). Length mixes of lane blocks only, up to 256 B,
    up to 1 KiB and the class edges, sometimes one block over 1 KiB (the general path then folds the
    batch); gapped, back-to-back, shuffled and overlapping layouts; base shifts; both polynomials.
    Every block against the oracle (CRC-32C sampled), and which kernel folded the batch."""
    rng = np.random.default_rng(9000 + seed + OFFSET)
    algo = ALGOS[seed % 2]
    n = int(rng.choice([262_144, 300_001, 400_003]))
    mix = ("lanes", "small", "mid", "edges")[seed // 2 % 4]
    if mix == "lanes":
        lens = rng.integers(0, 65, n)
    elif mix == "small":
        lens = rng.integers(0, 257, n)
    elif mix == "mid":
        lens = rng.integers(0, 1025, n)
    else:
        lens = rng.choice(np.array([0, 1, 3, 4, 63, 64, 65, 127, 128, 129, 255, 256, 257, 1023, 1024]), n)
    big = rng.random() < 0.25
    if big:
        lens[int(rng.integers(0, n))] = int(rng.integers(1025, 5000))
    layout = ("gapped", "back_to_back", "shuffled", "overlapping")[seed % 4]
    start = int(rng.integers(0, 64))
    if layout == "overlapping":
        offs = rng.integers(0, max(1, int(lens.sum()) // 3), n) + start
    else:
        gaps = rng.integers(0, 20, n) if layout != "back_to_back" else np.zeros(n, np.int64)
        offs = start + np.concatenate([[0], np.cumsum(lens + gaps)[:-1]])
        if layout == "shuffled":
            p = rng.permutation(n)
            offs, lens = offs[p], lens[p]
    host = rng.integers(0, 256, int((offs + lens).max()) + 64, dtype=np.uint8)
    shift = int(rng.integers(0, 16))
    d = on_device(host, gpu, shift)
    got = u32(tk.crc32_batch(d, torch.from_numpy(offs.astype(np.int64)).to(gpu),
                             torch.from_numpy(lens.astype(np.int32)).to(gpu), algo=algo))
    kp = tk.load_library().tkv_debug_irregular_path(ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    if big:
        assert kp == 2, (mix, layout)
    elif int(lens.max()) > 64:
        assert kp == 1, (mix, layout)
    else:
        assert kp in (0, 1), (mix, layout)  # (lane blocks whose first steps are no window take the packed mode)
    if algo == "crc32c":
        smp = rng.choice(n, 4000, replace=False)
        want = oracle_batch(oracle, algo, host, offs[smp], lens[smp], None)
        assert np.array_equal(got[smp], want), (mix, layout, shift)
        return
    want = oracle_batch(oracle, algo, host, offs, lens, None)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (f"{mix} {layout} n={n} shift={shift} path={kp}: {bad.size} differ, first {bad[:5]} "
                           f"(lens {lens[bad[:5]]})")
