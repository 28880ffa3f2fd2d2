"""TEST INFRASTRUCTURE ONLY (the checker, never the product): synthetic WAL images and their
sequential decode, for bench.py's post-timing `bit_exact_paths`, __graft_entry__.smoke() and tests/.

An image is a run of records laid out as wal_entry::encode writes them (/root/reference/src/engine/
wal.cpp:19-61; u32 record_len | u32 crc32 | u8 op | u64 seq | u8 tombstone | u32 key_len |
u32 value_len | key | value), stamped by oracle_wal_stamp (oracle/crc32_oracle.c, wal.cpp:54-58), so
nothing here depends on the product library. `decode` is oracle_wal_decode: engine::create's recovery
loop (engine.cpp:31-53) applying wal_entry::decode (wal.cpp:63-130) record after record.

Shapes (the ones VERDICT r5 names):
  small  - keys 4-23 B, values 0-39 B (WAL-put-sized records, 30-88 B each)
  zipf   - keys 8-63 B, values min(Zipf(1.6) * 64, 16000) B (long payloads beside short ones)
  values_of_records - every value is itself a run of well-formed 40-byte records (speculative
           header searches land on fake chains everywhere)
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
META = 26  # wal.hpp kMetadataSize


def load(path=None):
    o = ctypes.CDLL(path or os.path.join(HERE, "liboracle.so"))
    o.oracle_wal_stamp.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
    o.oracle_wal_decode.restype = ctypes.c_int
    o.oracle_wal_decode.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                    ctypes.POINTER(ctypes.c_uint64)]
    return o


def build(ora, klen, vlen, rng, fake_values=False):
    """Stamped image of records with key lengths `klen` and value lengths `vlen` (arrays): returns
    (image uint8, record offsets u64, record sizes u64). fake_values: every value is filled with as
    many whole well-formed 40-byte records (record_len 32, key 6, value 8) as fit."""
    klen = np.asarray(klen, np.uint64)
    vlen = np.asarray(vlen, np.uint64)
    n = klen.size
    size = META + klen + vlen
    offs = np.zeros(n, np.uint64)
    offs[1:] = np.cumsum(size[:-1])
    img = rng.integers(0, 256, int(size.sum()), dtype=np.uint8)
    hdr = np.zeros((n, META), np.uint8)
    hdr[:, 0:4] = (size - 8).astype("<u4").view(np.uint8).reshape(-1, 4)
    hdr[:, 9:17] = np.arange(n, dtype="<u8").view(np.uint8).reshape(-1, 8)
    hdr[:, 18:22] = klen.astype("<u4").view(np.uint8).reshape(-1, 4)
    hdr[:, 22:26] = vlen.astype("<u4").view(np.uint8).reshape(-1, 4)
    img[offs.astype(np.int64)[:, None] + np.arange(META)] = hdr
    if fake_values:
        fake = np.zeros(40, np.uint8)
        fake[0:4] = np.frombuffer((32).to_bytes(4, "little"), np.uint8)
        fake[18:22] = np.frombuffer((6).to_bytes(4, "little"), np.uint8)
        fake[22:26] = np.frombuffer((8).to_bytes(4, "little"), np.uint8)
        nb = (vlen // 40 * 40).astype(np.int64)  # bytes of fake records per value
        v0 = (offs + META + klen).astype(np.int64)
        tot = int(nb.sum())
        if tot:
            starts = np.repeat(v0, nb)
            within = np.arange(tot, dtype=np.int64) - np.repeat(np.cumsum(nb) - nb, nb)
            img[starts + within] = fake[within % 40]
    ora.oracle_wal_stamp(img.ctypes.data, offs.ctypes.data, n)
    return img, offs, size


def image(ora, shape, n, seed):
    rng = np.random.default_rng(seed)
    if shape == "small":
        return build(ora, rng.integers(4, 24, n), rng.integers(0, 40, n), rng)
    if shape == "zipf":
        return build(ora, rng.integers(8, 64, n), np.minimum(rng.zipf(1.6, n) * 64, 16000), rng)
    if shape == "values_of_records":
        return build(ora, rng.integers(0, 40, n), np.minimum(rng.zipf(1.6, n) * 48, 4000), rng, fake_values=True)
    raise ValueError(shape)


def decode(ora, img, size=None):
    """(status, n_good, stop_offset) of the sequential decode, as tkv_wal_verify reports them."""
    size = img.size if size is None else int(size)
    good, stop = ctypes.c_uint64(0), ctypes.c_uint64(0)
    bad = ora.oracle_wal_decode(img.ctypes.data if img.size else None, size, ctypes.byref(good), ctypes.byref(stop))
    return ("corrupted" if bad else "ok"), good.value, stop.value
