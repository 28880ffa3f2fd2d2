"""CPU tests of the WAL record-chain walk behind tkv_wal_verify (wal.cpp:63-87): the parallel,
speculative walk must return exactly the sequential walk's records, end and error flag, on clean
WALs, truncated/corrupted ones, records larger than a walker's piece, and WALs whose values are
themselves WAL records (decoys for the speculative starts)."""
import ctypes
import struct

import numpy as np
import pytest

import tinykvpp_amd as tk
from tinykvpp_amd.wal import encode_unstamped


def seq_chain(buf):
    """Reference semantics: while pos < size: need 26 bytes, then record_len + 8 <= remaining."""
    pos, out, n = 0, [], len(buf)
    while pos < n:
        if n - pos < 26:
            return out, pos, True
        (rlen,) = struct.unpack_from("<I", buf, pos)
        if rlen + 8 > n - pos:
            return out, pos, True
        out.append(pos)
        pos += 8 + rlen
    return out, pos, False


def lib_chain(buf):
    lib = tk.load_library()
    a = np.frombuffer(bytes(buf), np.uint8)
    cap = max(1, len(buf) // 26 + 1)
    out = np.zeros(cap, np.uint64)
    end, err = ctypes.c_uint64(), ctypes.c_int()
    n = lib.tkv_debug_wal_chain(ctypes.c_void_p(a.ctypes.data) if a.size else None, a.size,
                                ctypes.c_void_p(out.ctypes.data), cap, ctypes.byref(end), ctypes.byref(err))
    return [int(x) for x in out[:n]], end.value, bool(err.value)


def make_wal(rng, nbytes, max_value=4000, decoys=False):
    recs, total, seq = [], 0, 0
    while total < nbytes:
        k = rng.bytes(int(rng.integers(1, 40)))
        if decoys and rng.random() < 0.3:  # a value that is itself a run of WAL records
            v = b"".join(encode_unstamped(0, int(rng.integers(0, 1 << 40)), b"kk", rng.bytes(int(rng.integers(0, 90))), 0)
                         for _ in range(int(rng.integers(1, 6))))
        else:
            v = rng.bytes(int(min(rng.zipf(1.5) * 40, max_value)))
        r = encode_unstamped(int(rng.integers(0, 2)), seq, k, v, 0)
        recs.append(r)
        total += len(r)
        seq += 1
    return b"".join(recs)


@pytest.mark.parametrize("nbytes,decoys", [(0, False), (100, False), (20 << 20, False), (40 << 20, True)])
def test_chain_matches_sequential(nbytes, decoys):
    rng = np.random.default_rng(nbytes + decoys)
    w = make_wal(rng, nbytes, decoys=decoys) if nbytes else b""
    assert lib_chain(w) == seq_chain(w)


def test_chain_corruptions():
    rng = np.random.default_rng(3)
    w = bytearray(make_wal(rng, 48 << 20))
    assert lib_chain(w) == seq_chain(w)
    starts, _, _ = seq_chain(w)
    for victim in (len(starts) // 3, len(starts) // 2 + 7, len(starts) - 2):
        bad = bytearray(w)
        struct.pack_into("<I", bad, starts[victim], 0x7FFFFFF0)  # record_len past the end
        assert lib_chain(bad) == seq_chain(bad)
        shorter = bytearray(w)
        struct.pack_into("<I", shorter, starts[victim], 20)  # chain goes off the rails mid-WAL
        assert lib_chain(shorter) == seq_chain(shorter)
    assert lib_chain(w[:-5]) == seq_chain(w[:-5])  # truncated tail


def test_chain_huge_records():
    rng = np.random.default_rng(4)
    big = encode_unstamped(0, 1, b"big", rng.bytes(30 << 20), 0)  # spans several walker pieces
    w = make_wal(rng, 10 << 20) + big + make_wal(rng, 20 << 20)
    assert lib_chain(w) == seq_chain(w)
