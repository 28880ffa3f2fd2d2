"""Shared fixtures. `-m "not gpu"` runs everywhere (oracle, golden vectors, host logic, ABI
symbols); `-m gpu` needs an MI355X and calls the HIP kernels through the C ABI."""
import ctypes
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a GPU (MI355X); calls the HIP path through the C ABI")


def _loaded_objects(substr):
    """Shared objects of this process whose path contains `substr` (from /proc/self/maps)."""
    try:
        with open("/proc/self/maps") as f:
            return sorted({ln.split()[-1] for ln in f if substr in ln and ln.rstrip().endswith(".so")})
    except OSError:
        return []


def pytest_collection_finish(session):
    """A GPU session states, before any test runs, which product library it loaded (absolute path,
    as the dynamic loader mapped it) and which device architecture it runs on, so the record ties
    the parity results to the gfx950 build of tinykvpp_amd/libtkv_crc32.so."""
    if not any(item.get_closest_marker("gpu") for item in session.items):
        return
    tr = session.config.pluginmanager.get_plugin("terminalreporter")
    say = tr.write_line if tr is not None else print
    import torch
    import tinykvpp_amd
    from tinykvpp_amd import build_id
    tinykvpp_amd.load_library()
    libs = _loaded_objects("libtkv_crc32")
    say(f"[tkv] product library loaded: {', '.join(libs) or 'NOT MAPPED'}")
    lib_id, tree, same = build_id.check()
    say(f"[tkv] build id: library {lib_id}, tree sources {tree}: {'match' if same else 'MISMATCH'}")
    if not same:
        pytest.exit(f"libtkv_crc32.so (build {lib_id}) was not built from this tree's sources ({tree}); rebuild it",
                    returncode=3)
    if torch.cuda.is_available():
        p = torch.cuda.get_device_properties(0)
        say(f"[tkv] device 0: {p.name}, arch {getattr(p, 'gcnArchName', '?')}, "
            f"{p.multi_processor_count} CUs, {p.total_memory / 2**30:.0f} GiB; torch {torch.__version__}")
    else:
        say("[tkv] no GPU visible to torch")


def golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


class Oracle:
    """ctypes view of oracle/liboracle.so (TEST INFRASTRUCTURE: the checker, never the product)."""

    def __init__(self, path):
        o = ctypes.CDLL(path)
        o.oracle_update.restype = ctypes.c_uint32
        o.oracle_update.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
        o.oracle_crc32.restype = ctypes.c_uint32
        o.oracle_crc32.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        o.oracle_table.argtypes = [ctypes.c_void_p]
        o.oracle_splitmix64.restype = ctypes.c_uint64
        o.oracle_splitmix64.argtypes = [ctypes.c_uint64]
        o.oracle_fill.argtypes = [ctypes.c_uint64] * 3 + [ctypes.c_void_p, ctypes.c_size_t]
        o.oracle_crc_synthetic.argtypes = [ctypes.c_uint64] * 4 + [ctypes.c_void_p]
        o.oracle_zipf_lengths.argtypes = [ctypes.c_uint64] * 3 + [ctypes.c_void_p]
        o.oracle_crc_synthetic_lens.argtypes = [ctypes.c_uint64] * 3 + [ctypes.c_void_p, ctypes.c_void_p]
        o.oracle_crc_batch.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint64, ctypes.c_void_p]
        o.oracle_crc32c.restype = ctypes.c_uint32
        o.oracle_crc32c.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        o.oracle_update_c.restype = ctypes.c_uint32
        o.oracle_update_c.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
        o.oracle_table_c.argtypes = [ctypes.c_void_p]
        o.oracle_sst_stamp.restype = ctypes.c_uint32
        o.oracle_sst_stamp.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        self.lib = o

    def crc(self, data: bytes) -> int:
        a = np.frombuffer(bytes(data), np.uint8)
        return self.lib.oracle_crc32(a.ctypes.data if a.size else None, a.size)

    def crc_c(self, data: bytes) -> int:
        a = np.frombuffer(bytes(data), np.uint8)
        return self.lib.oracle_crc32c(a.ctypes.data if a.size else None, a.size)

    def update_c(self, raw: int, data: bytes) -> int:
        a = np.frombuffer(bytes(data), np.uint8)
        return self.lib.oracle_update_c(raw, a.ctypes.data if a.size else None, a.size)

    def sst_stamp(self, image: bytes) -> int:
        a = np.frombuffer(bytes(image), np.uint8)
        return self.lib.oracle_sst_stamp(a.ctypes.data, a.size)

    def update(self, raw: int, data: bytes) -> int:
        a = np.frombuffer(bytes(data), np.uint8)
        return self.lib.oracle_update(raw, a.ctypes.data if a.size else None, a.size)

    def fill(self, seed, block, off, n):
        out = np.zeros(n, np.uint8)
        self.lib.oracle_fill(seed, block, off, out.ctypes.data, n)
        return out

    def synthetic(self, seed, first, count, length):
        out = np.zeros(count, np.uint32)
        self.lib.oracle_crc_synthetic(seed, first, count, length, out.ctypes.data)
        return out

    def zipf_lengths(self, seed, first, count):
        out = np.zeros(count, np.uint64)
        self.lib.oracle_zipf_lengths(seed, first, count, out.ctypes.data)
        return out

    def synthetic_lens(self, seed, first, lens):
        lens = np.ascontiguousarray(lens, np.uint64)
        out = np.zeros(lens.size, np.uint32)
        self.lib.oracle_crc_synthetic_lens(seed, first, lens.size, lens.ctypes.data, out.ctypes.data)
        return out

    def batch(self, base: np.ndarray, offsets, lengths, init=None):
        off = np.ascontiguousarray(offsets, np.uint64)
        ln = np.ascontiguousarray(lengths, np.uint32)
        ini = None if init is None else np.ascontiguousarray(init, np.uint32)
        out = np.zeros(off.size, np.uint32)
        self.lib.oracle_crc_batch(base.ctypes.data, off.ctypes.data, ln.ctypes.data,
                                  None if ini is None else ini.ctypes.data, off.size, out.ctypes.data)
        return out


@pytest.fixture(scope="session")
def oracle():
    path = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(path):
        import subprocess
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all"], check=True)
    return Oracle(path)


@pytest.fixture(scope="session")
def ref_lib():
    """The reference's own crc32.cpp compiled by oracle/Makefile (absent on the GPU box unless built)."""
    path = os.path.join(ROOT, "oracle", "_ref", "libref_crc32.so")
    if not os.path.exists(path):
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    r = ctypes.CDLL(path)
    r.ref_crc32.restype = ctypes.c_uint32
    r.ref_crc32.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    return r


@pytest.fixture(scope="session")
def lib():
    import tinykvpp_amd
    return tinykvpp_amd.load_library()


@pytest.fixture(scope="session")
def gpu():
    import torch
    import tinykvpp_amd as tk
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but torch sees no GPU")
    torch.cuda.set_device(0)
    tk.set_device(0)
    return torch.device("cuda:0")


# ---- which path an irregular batch takes: the prepass's verdict restated --------
LANE_MAX = 64        # kLaneMax
GROUP_MAX = 256      # kGroupMax: blocks of LANE_MAX + 1 .. GROUP_MAX are group blocks
SMALL_MAX = 1024     # kSmallMax
SCAN_TILE = 4096     # kScanTile
GROUP_DENSE_TILE = 3072  # kGroupDenseTile
GROUP_TILE_ROWS = 1024   # kGroupTileRows
STREAM_SMALL_TILE = 1024  # kStreamSmallTile
LANE_DENSE_TILE = 256    # kLaneDenseTile
# group classes (lower bound exclusive, upper inclusive, tile threshold, phase bit): 4- and 8-lane passes
GROUP_CLASSES = ((LANE_MAX, 256, 3072, 2), (256, 512, 3968, 4))


def phases_expected(lens):
    """The general path's phase bits the prepass publishes (tkv_debug_irregular_phases): per scan tile
    of 4096 blocks, lane blocks (<= 64 B) when it holds at least 256 of them, and each group class when
    it holds at least that class's threshold and at most GROUP_TILE_ROWS rows of blocks over SMALL_MAX."""
    lens = np.asarray(lens, np.int64)
    ph = 0
    for t in range(0, lens.size, SCAN_TILE):
        tl = lens[t:t + SCAN_TILE]
        if np.count_nonzero(tl <= LANE_MAX) >= LANE_DENSE_TILE:
            ph |= 1
        big = tl[tl > SMALL_MAX]
        if int(((big - 1) // 4096 + 1).sum()) <= GROUP_TILE_ROWS:
            for lo, hi, thr, bit in GROUP_CLASSES:
                if np.count_nonzero((tl > lo) & (tl <= hi)) >= thr:
                    ph |= bit
    return ph


def lists_expected(lens):
    """The small-block lists the prepass builds (tkv_debug_irregular_lists) for a general-path batch:
    blocks of at most SMALL_MAX bytes that no lane or group pass takes (phases_expected's per-tile
    verdicts), and how many of them are at most 256 and 257-512 bytes."""
    lens = np.asarray(lens, np.int64)
    listed = []
    for t in range(0, lens.size, SCAN_TILE):
        tl = lens[t:t + SCAN_TILE]
        taken = np.zeros(tl.size, bool)
        if np.count_nonzero(tl <= LANE_MAX) >= LANE_DENSE_TILE:
            taken |= tl <= LANE_MAX
        big = tl[tl > SMALL_MAX]
        if int(((big - 1) // 4096 + 1).sum()) <= GROUP_TILE_ROWS:
            for lo, hi, thr, _ in GROUP_CLASSES:
                cls = (tl > lo) & (tl <= hi)
                if np.count_nonzero(cls) >= thr:
                    taken |= cls
        listed.append(tl[(tl <= SMALL_MAX) & ~taken])
    ls = np.concatenate(listed) if listed else np.zeros(0, np.int64)
    return (int(ls.size), int(np.count_nonzero(ls <= 256)), int(np.count_nonzero((ls > 256) & (ls <= 512))))


def stream_expected(offs, lens, group_stream=False):
    """1 when the prepass picks the byte-stream walk for this batch, else 0: every block at least
    LANE_MAX + 1 bytes and starting where its predecessor ends, and (unless tkv_debug_set_stream_groups
    is on) no scan tile whose bytes are mostly in small blocks (at least STREAM_SMALL_TILE blocks of at
    most SMALL_MAX bytes among its 4096, with at most GROUP_TILE_ROWS rows of larger blocks)."""
    offs = np.asarray(offs, np.int64)
    lens = np.asarray(lens, np.int64)
    if lens.size == 0 or lens.min() <= LANE_MAX or np.any(offs[:-1] + lens[:-1] != offs[1:]):
        return 0
    if group_stream:
        return 1
    for t in range(0, lens.size, SCAN_TILE):
        tl = lens[t:t + SCAN_TILE]
        small = int(np.count_nonzero(tl <= SMALL_MAX))
        big = tl[tl > SMALL_MAX]
        rows = int(((big - 1) // 4096 + 1).sum())
        if small >= STREAM_SMALL_TILE and rows <= GROUP_TILE_ROWS:
            return 0
    return 1


@pytest.fixture
def stream_groups():
    """Sets tkv_debug_set_stream_groups(1) for one test (group-dense back-to-back batches may take the
    byte-stream walk, as before round 4), so the walk's many-ends-per-row shapes stay under test."""
    import tinykvpp_amd as tk
    lib = tk.load_library()
    prev = lib.tkv_debug_set_stream_groups(1)
    yield
    lib.tkv_debug_set_stream_groups(prev)
