"""C-ABI library checks that need no GPU: exported symbols, constant tables, and a numpy model of
the exact kernel decomposition (rows, lanes, slicing-by-4, lane shifts, Horner, init injection,
seam fix-up, wave partition) checked against the oracle."""
import ctypes
import os
import re

import numpy as np
import pytest

import tinykvpp_amd as tk
from tinykvpp_amd._lib import SIGNATURES

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROW, SEG = 4096, 64
POLY = 0xEDB88320


def header_symbols():
    text = open(os.path.join(ROOT, "include", "tkv_crc32.h")).read()
    return sorted(set(re.findall(r"\b(tkv_\w+)\s*\(", text)))


def test_library_exports_every_header_symbol(lib):
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), f"libtkv_crc32.so does not export {s}"
    assert sorted(SIGNATURES) == syms, "ctypes signatures out of sync with include/tkv_crc32.h"


def test_no_gpu_is_an_error_not_a_fallback(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    assert lib.tkv_device_count() == 0
    with pytest.raises(tk.TkvError) as e:
        tk.crc32().update(b"123456789")
    assert e.value.code == 2  # io_error: no device, and no CPU path to fall back to


def test_record_check_arguments_without_a_gpu(lib):
    """tkv_wal_check_records_device: null pointers and images over 4 GiB (u32 offsets) are invalid
    arguments, checked before any device work; with valid arguments and no GPU it is an I/O error,
    never a CPU fallback."""
    import torch
    f = lib.tkv_wal_check_records_device
    dummy = ctypes.c_void_p(16)  # never dereferenced
    assert f(dummy, 100, dummy, 5, 64, None, None, None) == 3          # no first_bad
    assert f(None, 100, dummy, 5, 64, None, dummy, None) == 3          # no image
    assert f(dummy, (1 << 32) + 2, dummy, 5, 64, None, dummy, None) == 3  # over 4 GiB
    if not torch.cuda.is_available():
        assert f(dummy, 100, dummy, 5, 64, None, dummy, None) == 2       # io_error: no device


def test_oversize_irregular_batch_is_rejected(lib):
    """Irregular batches carry u32 block indices; a count the prepass cannot index (within one scan
    tile of 2^32) is an invalid argument, checked before any device work (no GPU needed)."""
    import ctypes
    f = lib.tkv_crc32_batch_device
    f.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_uint64, ctypes.c_void_p]
    dummy = ctypes.c_void_p(16)  # never dereferenced: the size check comes first
    for n in (0xFFFFFFFF, 0xFFFFFFFF - 8191, 1 << 40):
        assert f(dummy, dummy, dummy, None, dummy, n, None) == 3  # TKV_INVALID_ARGUMENT


def load_tables(lib, poly=0xEDB88320):
    n = lib.tkv_debug_tables_poly(poly, None, 0)
    buf = np.zeros(n // 4, np.uint32)
    lib.tkv_debug_tables_poly(poly, buf.ctypes.data, n)
    o = 0
    slice_ = buf[o:o + 1024].reshape(4, 256); o += 1024
    lane = buf[o:o + 8 * 16 * 64].reshape(8, 16, 64); o += 8 * 16 * 64
    horner = buf[o:o + 64]; o += 64
    row_pow = buf[o:o + 64]; o += 64
    head = buf[o:o + (ROW + 1) * 32].reshape(ROW + 1, 32); o += (ROW + 1) * 32
    rows_shift = buf[o:o + 4096]; o += 4096
    inv_shift = buf[o:o + ROW + 1]; o += ROW + 1
    # inv_shift[d] = x^(-8d): multiplying by x^(8d) (Shift_d of it) gives x^0 back
    if poly == POLY:  # the debug GF(2) helpers are the CRC-32 polynomial's
        for d in (0, 1, 3, 100, 4096):
            assert lib.tkv_debug_multmodp(lib.tkv_debug_x8nmodp(d), int(inv_shift[d])) == 0x80000000
    # rows_shift[k] = x^(8*4096*k): rows_shift[0] = x^0, [1] = row_pow[0], [2^k] = row_pow[k]
    assert int(rows_shift[0]) == 0x80000000
    for k in range(12):
        assert int(rows_shift[1 << k]) == int(buf[1024 + 8 * 16 * 64 + 64 + k])
    built_for = int(buf[o]); o += 3  # poly + 2 pad words
    init_shift = buf[o:o + 1025]; o += 1025  # [h] = Shift_h(0xFFFFFFFF): the group walks' init term
    if poly == POLY:
        for h in (0, 1, 65, 200, 256, 257, 300, 512, 513, 777, 1024):
            assert int(init_shift[h]) == lib.tkv_debug_multmodp(lib.tkv_debug_x8nmodp(h), 0xFFFFFFFF)
    # the group phase's result is init_shift[h] ^ crc_0(block) = crc_init(block) (affine start)
    assert o * 4 == n
    assert built_for == poly
    return slice_, lane, horner, row_pow, head


@pytest.fixture(scope="module")
def tables(lib):
    return load_tables(lib)


def shift_zeros(oracle, reg, n):
    """Shift_n(reg) computed the slow way: feed n zero bytes to the reference algorithm."""
    return oracle.update(reg, b"\0" * n)


def test_slice_tables(tables, oracle):
    from conftest import golden
    s = tables[0]
    assert [int(x) for x in s[0]] == golden("kat.json")["table"]
    for k in range(1, 4):  # Tk[i] = register after feeding k zero bytes from T0[i]
        for i in (0, 1, 77, 255):
            assert int(s[k][i]) == shift_zeros(oracle, int(s[0][i]), k)


def test_gf2_helpers(lib, oracle):
    rng = np.random.default_rng(3)
    for n in [0, 1, 3, 4, 64, 4032, 4096, 100000]:
        z = lib.tkv_debug_x8nmodp(n)
        for v in rng.integers(0, 2**32, 4, dtype=np.uint64):
            assert lib.tkv_debug_multmodp(z, int(v)) == shift_zeros(oracle, int(v), n)


def test_crc32c_tables(lib, oracle):
    """The Castagnoli tables obey the same identities under the CRC-32C oracle."""
    s, lane, horner, row_pow, head = load_tables(lib, 0x82F63B78)
    t = np.zeros(256, np.uint32)
    oracle.lib.oracle_table_c(t.ctypes.data)
    assert np.array_equal(s[0], t)
    zc = lambda reg, n: oracle.update_c(reg, b"\0" * n)  # noqa: E731
    for k in range(1, 4):
        assert int(s[k][77]) == zc(int(s[0][77]), k)
    for l in (0, 40, 63):
        assert int(lane[5][11][l]) == zc(11 << 20, (63 - l) * SEG)
    assert int(horner[9]) == zc(1 << 9, ROW)
    assert int(head[1234][30]) == zc(1 << 30, 1234)
    assert int(row_pow[1]) == zc(0x80000000, 2 * ROW)
    # the tables differ from the reference's: the polynomial really is a parameter
    assert not np.array_equal(s[0], load_tables(lib)[0][0])


def test_lane_shift_horner_head_tables(tables, oracle):
    _, lane, horner, row_pow, head = tables
    for l in (0, 1, 31, 62, 63):
        for j in (0, 3, 7):
            for v in (1, 9, 15):
                assert int(lane[j][v][l]) == shift_zeros(oracle, v << (4 * j), (63 - l) * SEG)
    for i in (0, 5, 31):
        assert int(horner[i]) == shift_zeros(oracle, 1 << i, ROW)
    assert all(int(x) == 0 for x in horner[32:])
    for h in (0, 1, 3, 4, 100, 4095, 4096):
        for i in (0, 17, 31):
            assert int(head[h][i]) == shift_zeros(oracle, 1 << i, h)


# ---- numpy model of the kernel ------------------------------------------------------------------

def rows_for_len(n):
    return 1 if n == 0 else (n - 1) // ROW + 1


def head_len(n):
    return n - (rows_for_len(n) - 1) * ROW


def bits_dot(sel, consts):
    """XOR of consts[i] over the set bits i of sel (the lane-parallel GF(2) product)."""
    out = 0
    for i in range(32):
        if (sel >> i) & 1:
            out ^= int(consts[i])
    return out


class Model:
    def __init__(self, tables):
        self.s, self.lane, self.horner, self.row_pow, self.head = tables

    def slice_lanes(self, row):
        """16 slicing-by-4 steps per lane over a (64, 64)-byte row image; returns (64,) partials."""
        dw = row.reshape(64, 16, 4).astype(np.uint32)
        dw = dw[..., 0] | (dw[..., 1] << 8) | (dw[..., 2] << 16) | (dw[..., 3] << 24)
        p = np.zeros(64, np.uint32)
        T = self.s
        for k in range(16):
            x = p ^ dw[:, k]
            p = T[3][x & 0xFF] ^ T[2][(x >> 8) & 0xFF] ^ T[1][(x >> 16) & 0xFF] ^ T[0][x >> 24]
        return p

    def row_value(self, row, B, init, head_row, h):
        p = self.slice_lanes(row)
        v = np.zeros(64, np.uint32)
        for j in range(8):
            v ^= self.lane[j][(p >> (4 * j)) & 15, np.arange(64)]
        acc = int(np.bitwise_xor.reduce(v))
        acc ^= bits_dot(B, self.horner[:32])
        if head_row:
            acc ^= bits_dot(init, self.head[h])
        return acc

    def row_image(self, data, n, r):
        R = rows_for_len(n)
        start = n - (R - r) * ROW
        img = np.zeros(ROW, np.uint8)
        lo = max(0, start)
        img[lo - start:] = data[lo:start + ROW]
        return img

    def block_pieces(self, data, init, cuts):
        """Partials of the row pieces [cuts[i], cuts[i+1]) of one block (seam emulation)."""
        n = len(data)
        h = head_len(n)
        out = []
        for a, b in zip(cuts[:-1], cuts[1:]):
            B = 0
            for r in range(a, b):
                B = self.row_value(self.row_image(data, n, r), B, init, r == 0, h)
            out.append((B, rows_for_len(n) - b))
        return out

    def crc(self, data, init=0xFFFFFFFF, cuts=None):
        R = rows_for_len(len(data))
        cuts = cuts or [0, R]
        acc = 0
        for partial, after in self.block_pieces(np.asarray(data, np.uint8), init, cuts):
            z = 0x80000000
            for k in range(64):
                if (after >> k) & 1:
                    z = tk.load_library().tkv_debug_multmodp(z, int(self.row_pow[k]))
            acc ^= tk.load_library().tkv_debug_multmodp(z, partial)
        return acc ^ 0xFFFFFFFF


@pytest.fixture(scope="module")
def model(tables):
    return Model(tables)


@pytest.mark.parametrize("n", [0, 1, 2, 3, 4, 5, 15, 16, 17, 63, 64, 65, 255, 1000, 4095, 4096, 4097,
                               8191, 8192, 12289])
def test_model_matches_oracle(model, oracle, n):
    rng = np.random.default_rng(n + 1)
    d = rng.integers(0, 256, n, dtype=np.uint8)
    for init in (0xFFFFFFFF, 0x0BADF00D):
        want = oracle.update(init, d.tobytes()) ^ 0xFFFFFFFF
        assert model.crc(d, init) == want


def test_model_seams(model, oracle):
    rng = np.random.default_rng(5)
    n = 5 * ROW + 123
    d = rng.integers(0, 256, n, dtype=np.uint8)
    want = oracle.crc(d.tobytes())
    for cuts in ([0, 1, 6], [0, 2, 3, 6], [0, 5, 6], [0, 1, 2, 3, 4, 5, 6]):
        assert model.crc(d, cuts=cuts) == want


def wave_partition(lengths, W):
    """Row partition of crc_rows + wave_start of rows_finish (irregular path), in Python."""
    rows = [rows_for_len(n) for n in lengths]
    rs = np.concatenate([[0], np.cumsum(rows)]).astype(np.int64)
    TR = int(rs[-1])
    starts = {}
    for b in range(len(lengths)):
        lo, hi = int(rs[b]), int(rs[b + 1])
        for w in range((lo * W + TR - 1) // TR, min(W, (hi * W + TR - 1) // TR)):
            starts[w] = b
    return rs, TR, starts


@pytest.mark.parametrize("W", [1, 16, 64, 4096])
def test_wave_start_partition(W):
    rng = np.random.default_rng(W)
    for trial in range(5):
        lengths = rng.integers(0, 40000, rng.integers(1, 200)).tolist()
        rs, TR, starts = wave_partition(lengths, W)
        for w in range(W):
            g0, g1 = w * TR // W, (w + 1) * TR // W
            if g0 < g1:
                b = starts[w]
                assert rs[b] <= g0 < rs[b + 1]


def test_model_small_block_groups(model, oracle):
    """crc_small's arithmetic (kSmallMax = 1 KiB): a block of n <= 1024 bytes right-aligned in a
    1 KiB mini-row, 16 lanes x 64 B, lane g shifted with the LS entry of lane 48 + g, and the init
    term spread over the group as two bits per lane with head_shift[n]."""
    rng = np.random.default_rng(12)
    for n in [0, 1, 3, 4, 17, 63, 64, 65, 500, 1023, 1024]:
        data = rng.integers(0, 256, n, dtype=np.uint8)
        init = int(rng.integers(0, 2**32))
        img = np.zeros(1024, np.uint8)
        img[1024 - n:] = data
        # the model's slicing runs on 64 lanes of 64 B: put the mini-row in lanes 48..63
        row = np.zeros(ROW, np.uint8)
        row[ROW - 1024:] = img
        p = model.slice_lanes(row)[48:]
        v = 0
        for g in range(16):
            for j in range(8):
                v ^= int(model.lane[j][(p[g] >> (4 * j)) & 15, 48 + g])
            v ^= bits_dot(init & (1 << g), model.head[n]) ^ bits_dot(init & (1 << (16 + g)), model.head[n])
        assert v ^ 0xFFFFFFFF == oracle.update(init, data.tobytes()) ^ 0xFFFFFFFF


def packed_small_group(n):
    """The slot kernels' G (crc_packed_small at n = 64 G, crc_packed_small_gen for other n): the smallest
    power of two with 64 G >= n (n <= 2048)."""
    g = 1
    while 64 * g < n:
        g *= 2
    return g


@pytest.mark.parametrize("n", [16, 48, 64, 80, 96, 128, 144, 256, 512, 1024, 1040, 2048])
def test_model_packed_small_slots(model, oracle, n):
    """The slot kernels' arithmetic on a wave row of 64/G uniform blocks of n bytes packed back to
    back: lane l of block l // G reads the 64 bytes at n - 64 G + 64 (l % G) of its
    block (pieces in front of the block read zeros), folds them, and moves the partial with the
    lane-shift column the workgroup copies into column l (device column 64 - G + l % G); the group's
    XOR plus Shift_n(init) is the raw register."""
    G = packed_small_group(n)
    bpr = 64 // G
    rng = np.random.default_rng(n)
    blocks = rng.integers(0, 256, (bpr, n), dtype=np.uint8)
    row = np.zeros(ROW, np.uint8)
    for lane in range(64):
        b, g = lane // G, lane % G
        off = n - 64 * G + 64 * g
        for i in range(4):  # the kernel's four 16-byte pieces: in front of the block -> zeros
            if off + 16 * i >= 0:
                row[64 * lane + 16 * i:64 * lane + 16 * i + 16] = blocks[b][off + 16 * i:off + 16 * i + 16]
    p = model.slice_lanes(row)
    col = np.array([64 - G + (lane % G) for lane in range(64)])  # fill_lds_group's column remap
    v = np.zeros(64, np.uint32)
    for j in range(8):
        v ^= model.lane[j][(p >> (4 * j)) & 15, col]
    init = 0xFFFFFFFF
    K = bits_dot(init, model.head[n])  # Shift_n(init): head_shift[n][i] = Shift_n(1 << i)
    for b in range(bpr):
        raw = int(np.bitwise_xor.reduce(v[b * G:(b + 1) * G])) ^ K
        assert raw ^ 0xFFFFFFFF == oracle.crc(blocks[b].tobytes()), (n, b)


def test_combine_matches_concatenation(lib, oracle):
    """tkv_crc32_combine / tkv_crc32c_combine (host arithmetic on 4-byte values, no device): the CRC
    of A || B from CRC(A), CRC(B), |B|, against zlib.crc32 and the oracle's CRC-32C of the
    concatenation; empty pieces included."""
    import zlib
    rng = np.random.default_rng(31)
    for la, lb in [(0, 0), (0, 5), (7, 0), (1, 1), (100, 3), (4096, 4097), (70000, 123457)]:
        a = rng.integers(0, 256, la, dtype=np.uint8).tobytes()
        b = rng.integers(0, 256, lb, dtype=np.uint8).tobytes()
        assert lib.tkv_crc32_combine(zlib.crc32(a), zlib.crc32(b), lb) == zlib.crc32(a + b)
        assert tk.crc32_combine(oracle.crc(a), oracle.crc(b), lb) == oracle.crc(a + b)
        assert (tk.crc32_combine(oracle.crc_c(a), oracle.crc_c(b), lb, algo="crc32c") ==
                oracle.crc_c(a + b))
    # lengths far beyond any buffer: Shift_n by square-and-multiply; Shift_m(Shift_n(x)) = Shift_(m+n)(x)
    x = 0x12345678
    n, m = (1 << 40) + 3, (1 << 33) + 11
    assert (lib.tkv_crc32_combine(lib.tkv_crc32_combine(x, 0, n), 0, m) ==
            lib.tkv_crc32_combine(x, 0, n + m))


def skewed_ranges(nblocks, G, skew=154):
    """Python restatement of crc_packed_body's SKEW partition (tkv_crc32_device.h): workgroup g gets
    blocks [g*n/G, (g+1)*n/G); its wave in slot k (class c = k // 4) a share ~ (skew/256)^c."""
    w = [256, skew, skew * skew // 256]
    w.append(w[2] * skew // 256)
    tot = 4 * sum(w)
    out = []
    for g in range(G):
        g0, gn = g * nblocks // G, (g + 1) * nblocks // G - g * nblocks // G
        for k in range(16):
            c, m = k >> 2, k & 3
            pre = 4 * sum(w[:c]) + m * w[c]
            b0 = g0 + gn * pre // tot
            out.append((b0, g0 + gn * (pre + w[c]) // tot - b0))
    return out


@pytest.mark.parametrize("nblocks,G", [(4096, 256), (262144, 256), (524288, 256), (5000, 7), (16, 1), (1000003, 304)])
def test_skewed_packed_partition_covers_batch(nblocks, G):
    """The skewed static partition of the packed kernel hands every block to exactly one wave, in
    order, and gives slot class 0 the largest share."""
    r = skewed_ranges(nblocks, G)
    pos = 0
    for b0, nb in r:
        assert b0 == pos and nb >= 0
        pos += nb
    assert pos == nblocks
    if nblocks >= 64 * G:
        first = r[:16]
        assert first[0][1] >= first[4][1] >= first[8][1] >= first[12][1]


def stream_row0(w, TR, W, skew=154):
    """Python restatement of dev::stream_row0 (tkv_crc32_device.h): first row of stream-mode wave w."""
    wt = [256, skew, skew * skew // 256]
    wt.append(wt[2] * skew // 256)
    tot = 4 * sum(wt)
    k = w & 15
    c, m = k >> 2, k & 3
    pre = 4 * sum(wt[:c]) + m * wt[c]
    g, G = w >> 4, W >> 4
    r0 = g * TR // G
    return r0 + ((g + 1) * TR // G - r0) * pre // tot


@pytest.mark.parametrize("TR,W", [(1, 16), (15, 16), (1327104, 4096), (1281, 4096), (5000, 4864), (99, 32)])
def test_stream_partition(TR, W):
    """Stream-mode waves cover the TR rows exactly once, in order (row0 nondecreasing, row0(W) = TR),
    and the prepass's binary search (stream_first_wave) finds the first wave at or after each row."""
    r0 = [stream_row0(w, TR, W) for w in range(W + 1)]
    assert r0[0] == 0 and r0[W] == TR
    assert all(a <= b for a, b in zip(r0, r0[1:]))
    import bisect
    for r in sorted({0, 1, TR // 3, TR - 1, TR} | set(range(0, TR + 1, max(1, TR // 97)))):
        lo, hi = 0, W
        while lo < hi:
            mid = (lo + hi) // 2
            if r0[mid] >= r:
                hi = mid
            else:
                lo = mid + 1
        assert lo == bisect.bisect_left(r0, r)
        if 0 < r <= TR:  # the wave holding row r-1 is the last one starting at or before it
            w = lo - 1
            assert r0[w] <= r - 1 < r0[w + 1]


def test_library_build_id_matches_tree(lib):
    """libtkv_crc32.so carries the hash of the sources it was built from (tinykvpp_amd/build_id.py,
    baked in by the Makefile); the in-tree library must be this tree's build."""
    from tinykvpp_amd import build_id
    lib_id, tree, same = build_id.check()
    assert len(tree) == 16 and same, f"library {lib_id} vs tree {tree}: rebuild with make -C tinykvpp_amd/csrc"


def lane_model(slice_, host, blk, n, init):
    """The lane kernels' arithmetic (lane_issue / lane_dwords / lane_fold): the 16-byte
    granules covering the block (clamped to its last granule), two selects by the start's dword offset,
    v_alignbyte by its byte offset, then slicing-by-4 from the block's own register over the whole
    dwords and Sarwate steps over the last n % 4 bytes."""
    al = blk & ~15
    last = (blk + n - 1) & ~15
    raw = []
    for i in range(5):
        p = al + 16 * i
        src = p if (n and p < last) else last
        raw += [int.from_bytes(bytes(host[src + 4 * j:src + 4 * j + 4]), "little") if n else 0 for j in range(4)]
    o = blk & 15
    if o & 8:
        raw = raw[2:] + [0, 0]
    if o & 4:
        raw = raw[1:] + [0]
    t = o & 3
    d = [((raw[k + 1] << 32 | raw[k]) >> (8 * t)) & 0xFFFFFFFF for k in range(16)]
    c = init
    for k in range(n >> 2):
        x = c ^ d[k]
        c = int(slice_[3][x & 255] ^ slice_[2][(x >> 8) & 255] ^ slice_[1][(x >> 16) & 255] ^ slice_[0][x >> 24])
    for j in range(n & 3):
        c = (c >> 8) ^ int(slice_[0][(c ^ (d[n >> 2] >> (8 * j))) & 255])
    return c


def test_model_lane_blocks(tables, oracle):
    rng = np.random.default_rng(45)
    host = rng.integers(0, 256, 4096, dtype=np.uint8)
    for n in list(range(0, 65)) + [36, 59, 26]:
        for blk in rng.integers(16, 4096 - 96, 6):
            init = int(rng.integers(0, 2**32))
            want = oracle.update(init, host[blk:blk + n].tobytes())
            assert lane_model(tables[0], host, int(blk), n, init) == want, (n, int(blk))
