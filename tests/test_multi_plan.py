"""The multi-device split of tkv_crc32_batch_host_multi, checked on CPU (no GPU needed).

SURVEY.md §8e: a host batch is split by bytes across the devices with no collective; a block of at
least 1 MiB that straddles a device's byte share is cut there and its pieces' 4-byte registers are
combined on the host (zlib's crc32_combine arithmetic). The planner and the combine step are exported
as tkv_debug_multi_plan / tkv_debug_multi_combine. Here the per-piece CRCs come from the test oracle
(what each device would return for its pieces), so the split and the recombination are verified
against the oracle's CRC of every whole block without any device: the device-side half is covered by
test_gpu_parity.py::test_host_multi_splits_large_blocks.
"""
import ctypes

import numpy as np
import pytest

SPLIT_MIN = 1 << 20
POLY, POLY_C = 0xEDB88320, 0x82F63B78
VP = ctypes.c_void_p


@pytest.fixture(scope="module")
def mlib(lib):
    lib.tkv_debug_multi_plan.restype = ctypes.c_size_t
    lib.tkv_debug_multi_plan.argtypes = [ctypes.c_int, VP, VP, VP, ctypes.c_uint64, VP, ctypes.c_size_t]
    lib.tkv_debug_multi_combine.argtypes = [ctypes.c_uint32, ctypes.c_int, VP, VP, VP, ctypes.c_uint64, VP, VP]
    return lib


def plan(mlib, ndev, offs, lens, init=None):
    offs = np.ascontiguousarray(offs, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint32)
    ini = None if init is None else np.ascontiguousarray(init, np.uint32)
    ip = None if ini is None else ini.ctypes.data
    k = mlib.tkv_debug_multi_plan(ndev, offs.ctypes.data, lens.ctypes.data, ip, offs.size, None, 0)
    rec = np.zeros((max(k, 1), 6), np.uint64)
    assert mlib.tkv_debug_multi_plan(ndev, offs.ctypes.data, lens.ctypes.data, ip, offs.size,
                                      rec.ctypes.data, k) == k
    return rec[:k]


def combine(mlib, poly, ndev, offs, lens, init, piece_final):
    offs = np.ascontiguousarray(offs, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint32)
    ini = None if init is None else np.ascontiguousarray(init, np.uint32)
    pf = np.ascontiguousarray(piece_final, np.uint32)
    out = np.zeros(offs.size, np.uint32)
    assert mlib.tkv_debug_multi_combine(poly, ndev, offs.ctypes.data, lens.ctypes.data,
                                        None if ini is None else ini.ctypes.data, offs.size, pf.ctypes.data,
                                        out.ctypes.data) == 0
    return out


def check_plan(rec, ndev, offs, lens, init):
    """Structural properties: device order, block order, exact cover of each block, cut rules."""
    offs = np.asarray(offs, np.uint64)
    lens = np.asarray(lens, np.uint64)
    n = offs.size
    assert np.all(np.diff(rec[:, 0].astype(np.int64)) >= 0), "pieces listed in device order"
    assert np.all(np.diff(rec[:, 1].astype(np.int64)) >= 0), "pieces in block order across devices"
    assert set(rec[:, 1].tolist()) == set(range(n)), "every block planned"
    total = int(lens.sum())
    dev_bytes = np.zeros(ndev, np.int64)
    for b in range(n):
        p = rec[rec[:, 1] == b]
        assert int(p[0, 5]) == 1 and all(int(h) == 0 for h in p[1:, 5]), "head flag on the first piece only"
        want_init = 0xFFFFFFFF if init is None else int(init[b])
        assert int(p[0, 4]) == want_init and all(int(x) == 0 for x in p[1:, 4]), "init on the head piece only"
        assert np.array_equal(p[:, 2], offs[b] + np.concatenate([[0], np.cumsum(p[:-1, 3])]).astype(np.uint64))
        assert int(p[:, 3].sum()) == int(lens[b]), "pieces cover the block exactly"
        if len(p) > 1:
            assert int(lens[b]) >= SPLIT_MIN, "only blocks of >= 1 MiB are cut"
            assert len(set(p[:, 0].tolist())) == len(p), "a cut block's pieces sit on distinct devices"
        for r in p:
            dev_bytes[int(r[0])] += int(r[3])
    # byte balance: device d ends within one uncut block of its share boundary
    uncut = max([int(lens[b]) for b in range(n) if len(rec[rec[:, 1] == b]) == 1] + [0])
    acc = np.cumsum(dev_bytes)
    for d in range(ndev - 1):
        assert abs(int(acc[d]) - total * (d + 1) // ndev) <= uncut
    return dev_bytes


def piece_finals(oracle, host, rec, algo):
    upd = oracle.update if algo == "crc32" else oracle.update_c
    return np.array([upd(int(r[4]), host[int(r[2]):int(r[2]) + int(r[3])].tobytes()) ^ 0xFFFFFFFF for r in rec],
                    np.uint32)


def whole(oracle, host, offs, lens, init, algo):
    upd = oracle.update if algo == "crc32" else oracle.update_c
    return np.array([upd(0xFFFFFFFF if init is None else int(init[b]), host[int(o):int(o) + int(l)].tobytes())
                     ^ 0xFFFFFFFF for b, (o, l) in enumerate(zip(offs, lens))], np.uint32)


@pytest.mark.parametrize("ndev", [1, 2, 3, 4, 8])
def test_small_blocks_split_by_index_ranges(mlib, ndev):
    rng = np.random.default_rng(ndev)
    lens = rng.integers(0, 70000, 5000).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.uint64)
    rec = plan(mlib, ndev, offs, lens)
    assert len(rec) == lens.size, "no block below 1 MiB is cut"
    dev_bytes = check_plan(rec, ndev, offs, lens, None)
    assert dev_bytes.max() - dev_bytes.min() <= 2 * 70000


@pytest.mark.parametrize("ndev", [2, 3, 4, 8])
@pytest.mark.parametrize("algo", ["crc32", "crc32c"])
def test_one_huge_block_spreads_over_devices(mlib, oracle, ndev, algo):
    rng = np.random.default_rng(40 + ndev)
    n = 9 << 20
    host = rng.integers(0, 256, n + 64, dtype=np.uint8)
    offs, lens = np.array([3], np.uint64), np.array([n], np.uint32)
    init = np.array([0x12345678], np.uint32)
    rec = plan(mlib, ndev, offs, lens, init)
    assert len(rec) == ndev and sorted(rec[:, 0].tolist()) == list(range(ndev))
    check_plan(rec, ndev, offs, lens, init)
    pf = piece_finals(oracle, host, rec, algo)
    got = combine(mlib, POLY if algo == "crc32" else POLY_C, ndev, offs, lens, init, pf)
    assert np.array_equal(got, whole(oracle, host, offs, lens, init, algo))


@pytest.mark.parametrize("ndev", [2, 3, 4, 5, 8])
def test_mixed_batch_with_cut_blocks(mlib, oracle, ndev):
    """Large blocks on share boundaries among small and empty ones, per-block initial registers,
    unordered offsets (blocks need not be laid out in index order in memory)."""
    rng = np.random.default_rng(90 + ndev)
    lens = np.array([(3 << 20) + 1, 0, (2 << 20) + 77, 100, 1 << 20, (4 << 20) - 3, 5, 0, (1 << 20) - 1, 7000],
                    np.uint32)
    offs = rng.permutation(np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64))])).astype(np.uint64)
    host = rng.integers(0, 256, int(lens.sum()) + (4 << 20), dtype=np.uint8)
    init = rng.integers(0, 1 << 32, lens.size, dtype=np.uint64).astype(np.uint32)
    rec = plan(mlib, ndev, offs, lens, init)
    check_plan(rec, ndev, offs, lens, init)
    assert len(rec) > lens.size, "some block straddles a share boundary and is cut"
    for algo in ("crc32", "crc32c"):
        pf = piece_finals(oracle, host, rec, algo)
        got = combine(mlib, POLY if algo == "crc32" else POLY_C, ndev, offs, lens, init, pf)
        assert np.array_equal(got, whole(oracle, host, offs, lens, init, algo))


def test_more_devices_than_blocks_and_empty_bytes(mlib, oracle):
    offs, lens = np.array([0, 0, 0], np.uint64), np.array([0, 0, 0], np.uint32)
    rec = plan(mlib, 8, offs, lens)
    check_plan(rec, 8, offs, lens, None)
    host = np.zeros(16, np.uint8)
    got = combine(mlib, POLY, 8, offs, lens, None, piece_finals(oracle, host, rec, "crc32"))
    assert np.array_equal(got, np.zeros(3, np.uint32))  # CRC of an empty block is 0
    lens2 = np.array([(1 << 20) + 5], np.uint32)
    rec2 = plan(mlib, 8, np.array([1], np.uint64), lens2)
    assert len(rec2) == 8 and int(rec2[:, 3].sum()) == int(lens2[0])
