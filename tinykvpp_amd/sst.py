"""SSTable data-block stamping and verification on the GPU CRC engine.

The reference leaves the checksum fields dead: get_data_block writes
``sstable_data_block_header::crc32_ = 0`` (/root/reference/src/storage/sstable_writer.cpp:138-144)
and read_data_block never checks it (sstable_reader.cpp:61-89). The format here is this library's
decision (include/tkv_crc32.h, "parity unpinned"): a data-block image, as get_data_block builds it
(sstable_writer.cpp:150-168), is

    varint(20) | header[20] | varint(n) | body[n] | padding up to 36 + n bytes

with header = u32 entry_count | u32 uncompressed_size | u32 compressed_size | u8 compression |
3 pad | u32 crc32_ (sstable_format.hpp:91-99), so crc32_ sits at image byte CRC_OFFSET = 17. The
stamp is crc32 over the whole image with those 4 bytes read as zero, stored little-endian.
"""
import ctypes
import struct

import numpy as np

from ._lib import CORRUPTED, OK, check, load_library

CRC_OFFSET = 17   # 1-byte varint(20) + 16 header bytes before crc32_
MIN_IMAGE = 22    # varint(20) + header + varint(0)


def _varint(v):
    """codec::encode_varint (core/serialization/codec.hpp:31-39): LEB128."""
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def encode_data_block_image(entries):
    """Unstamped image of a data block holding ``entries`` [(ikey, value), ...], laid out as
    sstable_writer::get_data_block does: the body is write_string(ikey) | write_string(value) per
    entry (sstable_writer.cpp:113) and the block size counts 4 + |ikey| + 4 + |value| per entry
    (:60,122); the reference leaves arena bytes in the slack past the written entries and in the
    image padding, which are zero here."""
    body = b"".join(_varint(len(k)) + k + _varint(len(v)) + v for k, v in entries)
    size = sum(8 + len(k) + len(v) for k, v in entries)
    body = body[:size].ljust(size, b"\0")
    header = struct.pack("<IIIB3xI", len(entries), size, size, 0, 0)
    image = _varint(len(header)) + header + _varint(size) + body
    return image.ljust(8 + len(header) + 8 + size, b"\0")


def _host_arrays(offsets, sizes):
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    sz = np.ascontiguousarray(sizes, dtype=np.uint64)
    if off.size != sz.size:
        raise ValueError("offsets and sizes differ in length")
    return off, sz


def stamp_blocks(file, offsets, sizes):
    """Stamp images in place in a writable uint8 numpy buffer (the SSTable file being written)."""
    if not isinstance(file, np.ndarray) or file.dtype != np.uint8 or not file.flags.writeable:
        raise ValueError("file must be a writable uint8 numpy array")
    off, sz = _host_arrays(offsets, sizes)
    check(load_library().tkv_sst_stamp_blocks(ctypes.c_void_p(file.ctypes.data), ctypes.c_void_p(off.ctypes.data),
                                              ctypes.c_void_p(sz.ctypes.data), off.size))


def verify_blocks(file, offsets, sizes):
    """Verify images of a host buffer. Returns (status, n_bad, first_bad); status "ok" or "corrupted"."""
    buf = np.ascontiguousarray(np.frombuffer(file, np.uint8) if not isinstance(file, np.ndarray) else file)
    off, sz = _host_arrays(offsets, sizes)
    n_bad, first = ctypes.c_uint64(0), ctypes.c_uint64(0)
    rc = load_library().tkv_sst_verify_blocks(ctypes.c_void_p(buf.ctypes.data), ctypes.c_void_p(off.ctypes.data),
                                              ctypes.c_void_p(sz.ctypes.data), off.size, ctypes.byref(n_bad),
                                              ctypes.byref(first))
    if rc not in (OK, CORRUPTED):
        check(rc)
    return ("ok" if rc == OK else "corrupted"), n_bad.value, first.value


def block_crcs_device(file, offsets, sizes, store=False, out=None, stream=None):
    """Device-resident images (torch uint8 CUDA tensor, int64 offsets, int32 sizes): the stamp value
    of every image (its CRC with the field read as zero); store=True also writes it into the field."""
    import torch
    from .crc32 import _check_data, _check_vec, _launch_stream, _out_vec
    n = offsets.numel()
    if sizes.numel() != n:
        raise ValueError("offsets and sizes differ in length")
    if file.dtype != torch.uint8:
        raise ValueError("file must be a uint8 tensor")
    _check_data(file)
    for name, t, dt in (("offsets", offsets, torch.int64), ("sizes", sizes, torch.int32)):
        _check_vec(name, t, dt, n, file.device)
    out = _out_vec(out, n, file.device, stream)
    check(load_library().tkv_sst_block_crcs_device(
        ctypes.c_void_p(file.data_ptr()), ctypes.c_void_p(offsets.data_ptr()), ctypes.c_void_p(sizes.data_ptr()),
        ctypes.c_void_p(out.data_ptr()), n, int(bool(store)), _launch_stream(stream, file.device)))
    return out


# ---- index image + footer (include/tkv_crc32.h "SSTable index image + footer stamping") ----------
FOOTER_SIZE = 20      # sizeof(sstable_footer) (sstable_format.hpp:129-135)
FOOTER_CRC_OFFSET = 16


def encode_index_image(entries):
    """Index image as sstable_writer::get_index lays it out: u64 entry count, then per entry
    write_string(smallest_key) | u64 data_block_offset | u64 data_block_size (write_string is
    varint length + bytes, buffer_writer.hpp:75-77). ``entries`` is [(smallest_key, offset, size)]."""
    out = bytearray(struct.pack("<Q", len(entries)))
    for key, off, size in entries:
        out += _varint(len(key)) + key + struct.pack("<QQ", off, size)
    return bytes(out)


def encode_footer(index_offset, index_size, bloom_offset=0, bloom_size=0):
    """Unstamped 20-byte footer in sstable_footer declaration order (crc32_ = 0)."""
    return struct.pack("<IIIII", index_offset, index_size, bloom_offset, bloom_size, 0)


def _index_ptr(index_image):
    buf = np.ascontiguousarray(np.frombuffer(index_image, np.uint8) if not isinstance(index_image, np.ndarray)
                               else index_image)
    return buf, buf.size


def stamp_footer(index_image, footer):
    """Stamped copy of ``footer`` (20 bytes): crc32_ = CRC-32 of index image || footer[0:16]."""
    if len(footer) != FOOTER_SIZE:
        raise ValueError("footer must be 20 bytes")
    idx, n = _index_ptr(index_image)
    f = (ctypes.c_uint8 * FOOTER_SIZE).from_buffer_copy(bytes(footer))
    check(load_library().tkv_sst_stamp_footer(ctypes.c_void_p(idx.ctypes.data if n else 0), n, f))
    return bytes(f)


def verify_footer(index_image, footer):
    """"ok" when the footer's crc32_ matches the index image and its own fields, else "corrupted"."""
    if len(footer) != FOOTER_SIZE:
        raise ValueError("footer must be 20 bytes")
    idx, n = _index_ptr(index_image)
    f = (ctypes.c_uint8 * FOOTER_SIZE).from_buffer_copy(bytes(footer))
    rc = load_library().tkv_sst_verify_footer(ctypes.c_void_p(idx.ctypes.data if n else 0), n, f)
    if rc not in (OK, CORRUPTED):
        check(rc)
    return "ok" if rc == OK else "corrupted"
