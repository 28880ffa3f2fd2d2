"""GPU parity of crc_packed_small_gen: uniform batches of blocks of 65 B - 2 KiB that
the exact slot kernel does not take - lengths that are not a multiple of 16, strides other than the
length (gapped, and overlapping blocks), base pointers at every alignment class, per-block initial
registers, CRC-32C - each block right-aligned in a slot of 64 G bytes folded by a G-lane group with
its granules realigned in registers. Everything is compared block by block with the oracle."""
import numpy as np
import pytest

import tinykvpp_amd as tk

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

LENGTHS = (65, 66, 100, 127, 128, 129, 200, 255, 256, 257, 300, 511, 513, 640, 1000, 1023, 1024, 1025,
           1500, 2000, 2047, 2048)


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def oracle_c(oracle, host, offs, n, init=None):
    out = np.zeros(len(offs), np.uint32)
    for i, o in enumerate(offs):
        raw = 0xFFFFFFFF if init is None else int(init[i])
        out[i] = oracle.update_c(raw, host[int(o):int(o) + n].tobytes()) ^ 0xFFFFFFFF
    return out


@pytest.fixture(scope="module")
def buf(gpu):
    rng = np.random.default_rng(2048)
    host = rng.integers(0, 256, (48 << 20) + 8192, dtype=np.uint8)
    return host, torch.from_numpy(host).to(gpu)


@pytest.mark.parametrize("blen", LENGTHS)
def test_uniform_small_any_shape(gpu, oracle, buf, blen):
    host, d = buf
    rng = np.random.default_rng(blen)
    g = 2
    while 64 * g < blen:
        g *= 2
    bpr = 64 // g
    # (stride, base offset, count): back to back at odd bases, gapped, overlapping; counts that end in a
    # partial wave row, single blocks, and batches large enough for every wave
    cases = [(blen, 1, 1), (blen, 3, bpr + 1), (blen + 8, 0, 4096 * bpr + 3), (blen + 3, 7, 5000),
             (max(1, blen - 5), 13, 3000), (blen, 0, 20000 // max(1, blen // 128)), (blen + 17, 6, 2 * bpr - 1)]
    for stride, off, n in cases:
        assert off + (n - 1) * stride + blen <= host.size
        offs = off + np.arange(n, dtype=np.uint64) * stride
        got = u32(tk.crc32_batch_uniform(d, blen, n, stride=stride, offset=off))
        want = oracle.batch(host, offs, np.full(n, blen, np.uint32))
        bad = np.flatnonzero(got != want)
        assert bad.size == 0, (stride, off, n, bad[:5])
        init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        it = torch.from_numpy(init.view(np.int32)).to(gpu)
        got = u32(tk.crc32_batch_uniform(d, blen, n, stride=stride, offset=off, init_raw=it))
        want = oracle.batch(host, offs, np.full(n, blen, np.uint32), init)
        bad = np.flatnonzero(got != want)
        assert bad.size == 0, ("init", stride, off, n, bad[:5])


@pytest.mark.parametrize("blen", (100, 257, 1025))
def test_uniform_small_crc32c(gpu, oracle, buf, blen):
    host, d = buf
    n, stride, off = 777, blen + 5, 9
    offs = off + np.arange(n, dtype=np.uint64) * stride
    got = u32(tk.crc32_batch_uniform(d, blen, n, stride=stride, offset=off, algo="crc32c"))
    assert np.array_equal(got, oracle_c(oracle, host, offs, blen))


def test_uniform_small_at_buffer_end(gpu, oracle):
    """The last block ends on the tensor's last byte (no granule past it may be read), at odd offsets."""
    rng = np.random.default_rng(5)
    for blen, n in ((65, 1000), (300, 333), (2047, 50)):
        for shift in (0, 1, 15):
            size = shift + n * blen
            host = rng.integers(0, 256, size, dtype=np.uint8)
            d = torch.from_numpy(host).to(gpu)
            got = u32(tk.crc32_batch_uniform(d, blen, n, offset=shift))
            offs = shift + np.arange(n, dtype=np.uint64) * blen
            assert np.array_equal(got, oracle.batch(host, offs, np.full(n, blen, np.uint32))), (blen, shift)
