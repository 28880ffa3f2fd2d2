"""tinykvpp_amd — MI355X-native CRC-32 block-checksum engine for tinykvpp's integrity path.

The product is libtkv_crc32.so (HIP kernels for gfx950 + C ABI, include/tkv_crc32.h). This package
is the Python mirror of the reference interface (frankie::core::crc32, crc32.hpp:32-49) and of the
WAL CRC call sites (wal.cpp:54-58, 89-96), over ctypes; plus SSTable block stamping (sst) and the
CRC-32C variant (crc32c), SURVEY.md §8f.
"""
from ._lib import TkvError, check, load_library  # noqa: F401
from .crc32 import (  # noqa: F401
    crc32,
    crc32_batch,
    crc32_batch_host,
    crc32_batch_uniform,
    crc32_combine,
    crc32c,
    device_count,
    fill_synthetic_blocks,
    fill_synthetic_uniform,
    generate_crc32_table,
    kCRC32Bits,
    kCRC32DefaultValue,
    kCRC32Polynomial,
    kCRC32TableSize,
    set_device,
)
from . import sst, wal  # noqa: F401
