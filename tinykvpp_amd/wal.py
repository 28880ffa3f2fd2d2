"""WAL record stamping and batched verification on the GPU CRC engine.

Mirrors the CRC call sites of frankie::engine::wal_entry (/root/reference/src/engine/wal.cpp):
  * encode (wal.cpp:19-61): record = u32 record_len | u32 crc32 | u8 op | u64 seq | u8 tombstone |
    u32 key_len | u32 value_len | key | value (LE, packed, 26-byte header, wal.hpp:21-27);
    record_len = size - 8; crc32 = crc32{}.update([8, size)).finalize() stored LE at offset 4.
  * decode (wal.cpp:63-130): eof on empty input; corrupted when fewer than 26 bytes remain, when
    record_len + 8 exceeds the input, on a CRC mismatch, or when key/value overflow the record.

Here a whole slurped WAL (wal_reader::open, wal.cpp:204-240) is verified on the GPU: the image is
copied to the device once, the record_len chain is walked there (speculative parallel walk with exact
stitching) and every record's CRC is checked in ONE batch (tkv_wal_verify; tkv_wal_verify_device for
an image already in HBM). Many records are stamped in one batch (tkv_wal_stamp) — the recovery loop
of engine::create (engine.cpp:31-53) and group commit.
"""
import ctypes
import struct

import numpy as np

from ._lib import CORRUPTED, OK, check, load_library

kMetadataSize = 26  # wal.hpp:21-27
PUT, DEL = 0, 1     # wal_operation (wal.hpp:14-17)


def encode_unstamped(op, seq, key, value, tombstone):
    """Record bytes laid out as wal.cpp:30-52 with the CRC field left zero (wal.cpp:28 memset)."""
    body = struct.pack("<BQBII", op, seq, int(bool(tombstone)), len(key), len(value)) + key + value
    return struct.pack("<II", len(body), 0) + body


def stamp(records):
    """Stamp a list of unstamped records (bytes) in one batch; returns the stamped bytes list."""
    if not records:
        return []
    sizes = np.array([len(r) for r in records], np.uint32)
    offs = np.zeros(len(records), np.uint64)
    offs[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
    buf = np.frombuffer(b"".join(records), np.uint8).copy()
    check(load_library().tkv_wal_stamp(ctypes.c_void_p(buf.ctypes.data), ctypes.c_void_p(offs.ctypes.data),
                                       ctypes.c_void_p(sizes.ctypes.data), len(records)))
    raw = buf.tobytes()
    return [raw[int(o):int(o) + int(s)] for o, s in zip(offs, sizes)]


def encode(op, seq, key, value, tombstone):
    """wal_entry::encode: one stamped record (uses the batch path with n = 1)."""
    return stamp([encode_unstamped(op, seq, key, value, tombstone)])[0]


def verify(wal_bytes):
    """Verify a slurped WAL image. Returns (status, n_good_records, stop_offset).

    status is "ok" (every record verified, clean eof) or "corrupted" (first bad record at
    stop_offset, the position wal_entry::decode leaves the view parked on, wal_test.cpp:809-850).
    """
    if isinstance(wal_bytes, np.ndarray):
        buf = np.ascontiguousarray(wal_bytes).reshape(-1).view(np.uint8)
    else:
        buf = np.frombuffer(wal_bytes, np.uint8)  # bytes / bytearray / memoryview: no copy
    good, stop = ctypes.c_uint64(0), ctypes.c_uint64(0)
    rc = load_library().tkv_wal_verify(ctypes.c_void_p(buf.ctypes.data) if buf.size else None, buf.size,
                                       ctypes.byref(good), ctypes.byref(stop))
    if rc not in (OK, CORRUPTED):
        check(rc)
    return ("ok" if rc == OK else "corrupted"), good.value, stop.value


def verify_device(image, size=None, stream=None):
    """Verify a WAL image held in a uint8 CUDA tensor (first ``size`` bytes; default all).
    Returns (status, n_good_records, stop_offset) as verify()."""
    import torch
    if image.dtype != torch.uint8 or not image.is_cuda or not image.is_contiguous():
        raise ValueError("image must be a contiguous uint8 CUDA tensor")
    n = image.numel() if size is None else int(size)
    if n > image.numel():
        raise ValueError("size exceeds the tensor")
    from .crc32 import _check_data, _launch_stream
    _check_data(image)  # the library's WAL scratch and tables are the current device's
    st = _launch_stream(stream, image.device)
    good, stop = ctypes.c_uint64(0), ctypes.c_uint64(0)
    rc = load_library().tkv_wal_verify_device(ctypes.c_void_p(image.data_ptr()), n, ctypes.byref(good),
                                              ctypes.byref(stop), st)
    if rc not in (OK, CORRUPTED):
        check(rc)
    return ("ok" if rc == OK else "corrupted"), good.value, stop.value


def check_records_device(image, rec_offsets, max_payload=64, crc_out=None, first_bad=None, stream=None):
    """wal_entry::decode's per-record checks (wal.cpp:63-127) for records whose starts are known:
    ``image`` a uint8 CUDA tensor, ``rec_offsets`` an int32/uint32 CUDA tensor of record start offsets
    (u32; images up to 4 GiB). Returns (first_bad, crc): first_bad is a 1-element int64 CUDA tensor
    holding the index of the first record that fails (len(rec_offsets) when none), crc an int32 CUDA
    tensor of each payload's computed CRC (``crc_out`` if given). Asynchronous on ``stream``, like a
    torch op issued there (tkv_wal_check_records_device)."""
    import torch
    from .crc32 import _check_data, _check_vec, _launch_stream
    if image.dtype != torch.uint8:
        raise ValueError("image must be a uint8 tensor (its size in bytes is its numel)")
    _check_data(image)
    n = rec_offsets.numel()
    if rec_offsets.dtype not in (torch.int32,):
        raise ValueError("rec_offsets must be an int32 tensor (u32 offsets)")
    _check_vec("rec_offsets", rec_offsets, torch.int32, n, image.device)
    # outputs allocated here are tied to a non-current stream for the caching allocator (as _out_vec)
    other = stream is not None and stream != torch.cuda.current_stream(image.device)
    if crc_out is None:
        crc_out = torch.empty(n, dtype=torch.int32, device=image.device)
        if other:
            crc_out.record_stream(stream)
    _check_vec("crc_out", crc_out, torch.int32, n, image.device)
    if first_bad is None:
        first_bad = torch.empty(1, dtype=torch.int64, device=image.device)
        if other:
            first_bad.record_stream(stream)
    _check_vec("first_bad", first_bad, torch.int64, 1, image.device)
    check(load_library().tkv_wal_check_records_device(
        ctypes.c_void_p(image.data_ptr()), image.numel(), ctypes.c_void_p(rec_offsets.data_ptr()), n,
        int(max_payload), ctypes.c_void_p(crc_out.data_ptr()), ctypes.c_void_p(first_bad.data_ptr()),
        _launch_stream(stream, image.device)))
    return first_bad, crc_out


def decode_fields(rec):
    """Header fields of one record (no checking): (record_len, crc, op, seq, tomb, key, value)."""
    record_len, crc = struct.unpack_from("<II", rec, 0)
    op, seq, tomb, klen, vlen = struct.unpack_from("<BQBII", rec, 8)
    key = rec[kMetadataSize:kMetadataSize + klen]
    value = rec[kMetadataSize + klen:kMetadataSize + klen + vlen]
    return record_len, crc, op, seq, tomb, key, value
