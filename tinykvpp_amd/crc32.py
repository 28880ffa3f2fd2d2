"""Python mirror of frankie::core::crc32 and the batch engine behind it.

Reference interface (/root/reference/src/core/crc32.hpp:9-49, crc32.cpp:9-22):

    constexpr kCRC32DefaultValue = 0xFFFFFFFF, kCRC32Bits = 8, kCRC32Polynomial = 0xEDB88320
    generate_crc32_table() -> std::array<uint32_t, 256>
    class crc32 { update(span<const byte>) -> crc32&; finalize() -> uint32_t; reset(); }

Same names, argument meaning and semantics here: ``crc32().update(b"...").finalize()``. Every
``update`` runs on the GPU through the C ABI (include/tkv_crc32.h); there is no CPU fallback.
The batch functions take torch tensors already resident on the GPU (or numpy arrays for the host
pipeline) and return ``finalize()`` values per block.
"""
import ctypes

import numpy as np

from ._lib import check, load_library

kCRC32DefaultValue = 0xFFFFFFFF  # crc32.hpp:9
kCRC32Bits = 8                   # crc32.hpp:10
kCRC32Polynomial = 0xEDB88320    # crc32.hpp:11
kCRC32TableSize = 256            # crc32.hpp:13


def generate_crc32_table():
    """The 256-entry Sarwate table (crc32.hpp:16-30); kept for API parity, not used to compute."""
    table = []
    for i in range(kCRC32TableSize):
        c = i
        for _ in range(kCRC32Bits):
            c = (c >> 1) ^ (kCRC32Polynomial if c & 1 else 0)
        table.append(c)
    return table


def _stream_ptr(stream):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def _launch_stream(stream, device):
    """The stream a batch launches on, ordered after the current stream's prior work: the inputs were
    written there, and the caching allocator may hand out an `out` block whose previous owner's
    kernels are still queued there (record_stream only guards the later free)."""
    import torch
    cur = torch.cuda.current_stream(device)
    if stream is not None and stream != cur:
        stream.wait_stream(cur)
    return ctypes.c_void_p((stream if stream is not None else cur).cuda_stream)


def _host_view(data):
    """(pointer, nbytes, keepalive) for a bytes-like or numpy host buffer."""
    if isinstance(data, np.ndarray):
        arr = np.ascontiguousarray(data)
        return arr.ctypes.data, arr.nbytes, arr
    mv = memoryview(data).cast("B")
    if mv.readonly:
        buf = ctypes.create_string_buffer(mv.tobytes(), len(mv))
        return ctypes.addressof(buf), len(mv), buf
    arr = np.frombuffer(mv, dtype=np.uint8)
    return arr.ctypes.data, arr.nbytes, arr


def _fn(algo, name):
    """C ABI entry ``tkv_<algo>_<name>`` (algo: "crc32" = the reference's CRC, "crc32c")."""
    if algo not in ("crc32", "crc32c"):
        raise ValueError(f"unknown checksum family {algo!r}")
    return getattr(load_library(), f"tkv_{algo}_{name}")


class crc32:  # noqa: N801 - reference class name (crc32.hpp:32)
    """CRC-32/ISO-HDLC accumulator; raw register starts at 0xFFFFFFFF (crc32.hpp:48)."""

    __slots__ = ("_crc",)
    _algo = "crc32"

    def __init__(self):
        self._crc = kCRC32DefaultValue

    def update(self, data, stream=None):
        """Continue the register over ``data`` (crc32.cpp:9-16) and return self (chainable).

        ``data``: bytes-like / numpy (host memory) or a torch uint8 tensor (device memory). The device
        kernel runs on ``stream`` (default: the current stream) after the current stream's prior
        work, and this call waits for its 4-byte result.
        """
        try:
            import torch
            is_dev = isinstance(data, torch.Tensor) and data.is_cuda
        except ImportError:  # pragma: no cover - torch is part of the image
            is_dev = False
        if is_dev:
            # the library launches on the current device, so the tensor must be there; a strided view
            # is checksummed over its elements in order, as a contiguous copy
            if data.device.index != torch.cuda.current_device():
                raise ValueError(f"data is on {data.device}, but the current device is "
                                 f"cuda:{torch.cuda.current_device()}")
            cur = torch.cuda.current_stream(data.device)
            t = data.contiguous().view(-1).view(torch.uint8)  # any copy runs on the current stream
            out = torch.empty(1, dtype=torch.int32, device=t.device)
            s = stream if stream is not None else cur
            if s != cur:
                s.wait_stream(cur)  # the kernel on `s` must see the bytes the current stream wrote
            check(_fn(self._algo, "update_device")(self._crc, ctypes.c_void_p(t.data_ptr()), t.numel(),
                                                   ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(s.cuda_stream)))
            s.synchronize()  # the 4-byte result is read below, after the kernel on `s` has written it
            self._crc = int(out.cpu().numpy().view(np.uint32)[0])
        else:
            ptr, n, keep = _host_view(data)
            res = ctypes.c_uint32(0)
            check(_fn(self._algo, "update")(self._crc, ctypes.c_void_p(ptr), n, ctypes.byref(res)))
            del keep
            self._crc = res.value
        return self

    def finalize(self):
        """Register XOR 0xFFFFFFFF (crc32.cpp:19)."""
        return self._crc ^ kCRC32DefaultValue

    def reset(self):
        """Back to 0xFFFFFFFF (crc32.cpp:22)."""
        self._crc = kCRC32DefaultValue

    @property
    def raw(self):
        return self._crc


class crc32c(crc32):  # noqa: N801
    """CRC-32C (Castagnoli, reflected 0x82F63B78, init/xorout 0xFFFFFFFF; RFC 3720 §B.4) on the same
    engine: SURVEY.md §8f rank 4, a format-versioned alternative, not reference behaviour."""

    __slots__ = ()
    _algo = "crc32c"


# ---- batch engine -------------------------------------------------------------------------------

def _u32_view(t):
    import torch
    return t.view(torch.int32) if t.dtype != torch.int32 else t


def _check_data(data):
    import torch
    if not isinstance(data, torch.Tensor) or not data.is_cuda or not data.is_contiguous():
        raise ValueError("data must be a contiguous CUDA tensor")
    if data.device.index != torch.cuda.current_device():
        raise ValueError(f"data is on {data.device}, but the current device is cuda:{torch.cuda.current_device()}")


def _check_vec(name, t, dtype, n, device):
    """A per-block vector: contiguous, of `dtype`, on the data's device, with at least n entries."""
    if not t.is_cuda or t.device != device or t.dtype != dtype or not t.is_contiguous() or t.numel() < n:
        raise ValueError(f"{name} must be a contiguous {dtype} tensor on {device} with >= {n} entries")


def _out_vec(out, n, device, stream):
    """The result vector: allocated here (and tied to `stream` for the caching allocator) or checked."""
    import torch
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=device)
        if stream is not None and stream != torch.cuda.current_stream(device):
            out.record_stream(stream)
        return out
    _check_vec("out", out, torch.int32, n, device)
    return out


def crc32_batch(data, offsets, lengths, init_raw=None, out=None, stream=None, algo="crc32"):
    """Irregular batch on the GPU: block i = data[offsets[i] : offsets[i] + lengths[i]].

    data: uint8 CUDA tensor; offsets: int64 CUDA tensor; lengths: int32 CUDA tensor (< 2^32 bytes
    each); init_raw: optional int32 CUDA tensor of raw registers (crc32::crc_). Returns an int32
    tensor of finalize() bit patterns (``.cpu().numpy().view(np.uint32)`` for unsigned values).
    Shapes, dtypes and devices are checked here; the block ranges themselves are trusted, as at the
    C ABI (include/tkv_crc32.h): every [offsets[i], offsets[i] + lengths[i]) must lie inside `data`.
    The kernels run on ``stream`` (default: the current stream) and the result is ready when that
    stream reaches this point, like any torch op issued on it.
    """
    import torch
    n = offsets.numel()
    if lengths.numel() != n:
        raise ValueError("offsets and lengths differ in length")
    _check_data(data)
    for name, t, dt in (("offsets", offsets, torch.int64), ("lengths", lengths, torch.int32)):
        _check_vec(name, t, dt, n, data.device)
    out = _out_vec(out, n, data.device, stream)
    if init_raw is not None:
        _check_vec("init_raw", init_raw, torch.int32, n, data.device)
    initp = ctypes.c_void_p(init_raw.data_ptr()) if init_raw is not None else None
    check(_fn(algo, "batch_device")(
        ctypes.c_void_p(data.data_ptr()), ctypes.c_void_p(offsets.data_ptr()),
        ctypes.c_void_p(lengths.data_ptr()), initp, ctypes.c_void_p(out.data_ptr()), n,
        _launch_stream(stream, data.device)))
    return out


def crc32_batch_uniform(data, length, n, stride=None, init_raw=None, out=None, stream=None, offset=0,
                        algo="crc32"):
    """Uniform batch on the GPU: block i = data[offset + i*stride : + length] (stride = length)."""
    import torch
    stride = length if stride is None else stride
    _check_data(data)
    if n and offset + (n - 1) * stride + length > data.numel():
        raise ValueError("batch exceeds the data tensor")
    out = _out_vec(out, n, data.device, stream)
    if init_raw is not None:
        _check_vec("init_raw", init_raw, torch.int32, n, data.device)
    initp = ctypes.c_void_p(init_raw.data_ptr()) if init_raw is not None else None
    check(_fn(algo, "batch_uniform_device")(
        ctypes.c_void_p(data.data_ptr() + offset), stride, length, initp,
        ctypes.c_void_p(out.data_ptr()), n, _launch_stream(stream, data.device)))
    return out


def crc32_batch_host(data, offsets, lengths, init_raw=None, devices=None, algo="crc32"):
    """Host-memory batch (numpy): pinned staging, H2D / kernel / D2H overlapped. Returns uint32."""
    buf = np.ascontiguousarray(data).view(np.uint8)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    ini = None if init_raw is None else np.ascontiguousarray(init_raw, dtype=np.uint32)
    out = np.zeros(off.size, np.uint32)
    initp = None if ini is None else ctypes.c_void_p(ini.ctypes.data)
    if devices is None:
        check(_fn(algo, "batch_host")(ctypes.c_void_p(buf.ctypes.data), ctypes.c_void_p(off.ctypes.data),
                                      ctypes.c_void_p(ln.ctypes.data), initp,
                                      ctypes.c_void_p(out.ctypes.data), off.size))
    else:
        devs = (ctypes.c_int * len(devices))(*devices)
        check(_fn(algo, "batch_host_multi")(devs, len(devices), ctypes.c_void_p(buf.ctypes.data),
                                             ctypes.c_void_p(off.ctypes.data), ctypes.c_void_p(ln.ctypes.data),
                                             initp, ctypes.c_void_p(out.ctypes.data), off.size))
    return out


def crc32_combine(crc1, crc2, len2, algo="crc32"):
    """CRC of A || B from CRC(A), CRC(B) and len(B) (zlib's crc32_combine; tkv_crc32_combine)."""
    return int(_fn(algo, "combine")(crc1, crc2, len2))


def fill_synthetic_uniform(data, length, n, first_block=0, seed=1, stride=None, stream=None):
    """Write the SURVEY §8d generator's blocks [first_block, first_block+n) into ``data`` (GPU)."""
    stride = length if stride is None else stride
    check(load_library().tkv_fill_synthetic_uniform(ctypes.c_void_p(data.data_ptr()), stride, length,
                                                    first_block, n, seed, _stream_ptr(stream)))


def fill_synthetic_blocks(data, offsets, lengths, first_block=0, seed=1, stream=None):
    check(load_library().tkv_fill_synthetic_blocks(ctypes.c_void_p(data.data_ptr()),
                                                   ctypes.c_void_p(offsets.data_ptr()),
                                                   ctypes.c_void_p(lengths.data_ptr()), first_block,
                                                   offsets.numel(), seed, _stream_ptr(stream)))


def device_count():
    return load_library().tkv_device_count()


def set_device(device):
    check(load_library().tkv_set_device(device))
