"""ctypes binding of libtkv_crc32.so (the C ABI declared in include/tkv_crc32.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (hipcc, gfx950). There is no
Python or CPU fallback for the checksum: if the library is missing, importing the compute entry
points raises, so a GPU run can never silently compute somewhere else.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libtkv_crc32.so")

# status codes: frankie::core::status_code (/root/reference/src/core/status.hpp:11-20)
STATUS = {0: "ok", 1: "not_found", 2: "io_error", 3: "invalid_argument", 4: "corrupted", 5: "eof",
          6: "out_of_memory", 7: "buffer_overflow"}
OK, NOT_FOUND, IO_ERROR, INVALID_ARGUMENT, CORRUPTED, EOF, OUT_OF_MEMORY, BUFFER_OVERFLOW = range(8)


class TkvError(RuntimeError):
    """A non-ok status from the C ABI (code mirrors frankie::core::status_code)."""

    def __init__(self, code, msg):
        super().__init__(f"{STATUS.get(code, code)}: {msg}")
        self.code = code


_u8p = ctypes.c_void_p
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
_int = ctypes.c_int

# name -> (restype, argtypes); must match include/tkv_crc32.h
SIGNATURES = {
    "tkv_device_count": (_int, []),
    "tkv_set_device": (_int, [_int]),
    "tkv_last_error": (ctypes.c_char_p, []),
    "tkv_build_id": (ctypes.c_char_p, []),
    "tkv_crc32_update": (_int, [_u32, _vp, _sz, ctypes.POINTER(_u32)]),
    "tkv_crc32_update_host": (_int, [_u32, _vp, _sz, ctypes.POINTER(_u32)]),
    "tkv_crc32c_update_host": (_int, [_u32, _vp, _sz, ctypes.POINTER(_u32)]),
    "tkv_crc32_update_fallback": (_int, [_int, _u32, _vp, _sz, ctypes.POINTER(_u32)]),
    "tkv_crc32c_update_fallback": (_int, [_int, _u32, _vp, _sz, ctypes.POINTER(_u32)]),
    "tkv_crc32_update_device": (_int, [_u32, _vp, _sz, _vp, _vp]),
    "tkv_crc32_batch_device": (_int, [_u8p, _vp, _vp, _vp, _vp, _u64, _vp]),
    "tkv_crc32_batch_uniform_device": (_int, [_u8p, _u64, _u64, _vp, _vp, _u64, _vp]),
    "tkv_crc32_batch_host": (_int, [_u8p, _vp, _vp, _vp, _vp, _u64]),
    "tkv_crc32_batch_host_multi": (_int, [_vp, _int, _u8p, _vp, _vp, _vp, _vp, _u64]),
    "tkv_crc32_combine": (_u32, [_u32, _u32, _u64]),
    "tkv_wal_verify": (_int, [_u8p, _u64, ctypes.POINTER(_u64), ctypes.POINTER(_u64)]),
    "tkv_wal_verify_device": (_int, [_u8p, _u64, ctypes.POINTER(_u64), ctypes.POINTER(_u64), _vp]),
    "tkv_wal_stamp": (_int, [_u8p, _vp, _vp, _u64]),
    "tkv_wal_check_records_device": (_int, [_u8p, _u64, _vp, _u64, _u32, _vp, _vp, _vp]),
    "tkv_fill_synthetic_uniform": (_int, [_u8p, _u64, _u64, _u64, _u64, _u64, _vp]),
    "tkv_fill_synthetic_blocks": (_int, [_u8p, _vp, _vp, _u64, _u64, _u64, _vp]),
    "tkv_sst_stamp_blocks": (_int, [_u8p, _vp, _vp, _u64]),
    "tkv_sst_verify_blocks": (_int, [_u8p, _vp, _vp, _u64, ctypes.POINTER(_u64), ctypes.POINTER(_u64)]),
    "tkv_sst_block_crcs_device": (_int, [_u8p, _vp, _vp, _vp, _u64, _int, _vp]),
    "tkv_sst_stamp_footer": (_int, [_u8p, _u64, _vp]),
    "tkv_sst_verify_footer": (_int, [_u8p, _u64, _vp]),
    "tkv_crc32c_update": (_int, [_u32, _vp, _sz, ctypes.POINTER(_u32)]),
    "tkv_crc32c_update_device": (_int, [_u32, _vp, _sz, _vp, _vp]),
    "tkv_crc32c_batch_device": (_int, [_u8p, _vp, _vp, _vp, _vp, _u64, _vp]),
    "tkv_crc32c_batch_uniform_device": (_int, [_u8p, _u64, _u64, _vp, _vp, _u64, _vp]),
    "tkv_crc32c_batch_host": (_int, [_u8p, _vp, _vp, _vp, _vp, _u64]),
    "tkv_crc32c_batch_host_multi": (_int, [_vp, _int, _u8p, _vp, _vp, _vp, _vp, _u64]),
    "tkv_crc32c_combine": (_u32, [_u32, _u32, _u64]),
    "tkv_debug_tables": (_sz, [_vp, _sz]),
    "tkv_debug_tables_poly": (_sz, [_u32, _vp, _sz]),
    "tkv_debug_multmodp": (_u32, [_u32, _u32]),
    "tkv_debug_x8nmodp": (_u32, [_u64]),
    "tkv_debug_set_host_mapped": (_int, [_int]),
    "tkv_debug_set_stream_groups": (_int, [_int]),
    "tkv_debug_set_one_pass": (_int, [_int]),
    "tkv_debug_wal_chain": (_sz, [_u8p, _u64, _vp, _sz, ctypes.POINTER(_u64), ctypes.POINTER(_int)]),
    "tkv_debug_wal_last": (None, [_vp]),
    "tkv_debug_wal_rounds": (ctypes.c_size_t, [_vp, ctypes.c_size_t]),
    "tkv_debug_update_counts": (None, [_vp]),
    "tkv_debug_update_counts_n": (_sz, [_vp, _sz]),
    "tkv_debug_irregular_mode": (_int, [_vp]),
    "tkv_debug_irregular_phases": (_int, [_vp]),
    "tkv_debug_irregular_path": (_int, [_vp]),
    "tkv_debug_list_lanes_waves": (ctypes.c_uint32, [ctypes.c_uint64]),
    "tkv_debug_irregular_lists": (_int, [_vp, _vp]),
    "tkv_debug_multi_plan": (_sz, [_int, _vp, _vp, _vp, _u64, _vp, _sz]),
    "tkv_debug_multi_combine": (_int, [_u32, _int, _vp, _vp, _vp, _u64, _vp, _vp]),
}

# symbols an older build may lack (tools/ab_lib.py loads earlier builds for A/B runs)
OPTIONAL = {"tkv_build_id"}

_lib = None


def load_library(path=LIB_PATH):
    """Load (once) and return the ctypes handle; raises if the HIP library was not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"{path} is missing: the HIP extension was not built "
                          "(run `python -c 'import __graft_entry__ as g; g.build()'`)")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        if name in OPTIONAL and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc):
    """Raise TkvError for a non-zero status, with the thread's last error text."""
    if rc != OK:
        raise TkvError(rc, load_library().tkv_last_error().decode(errors="replace"))
    return rc
