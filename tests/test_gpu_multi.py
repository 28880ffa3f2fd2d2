"""The multi-device split on the GPU, piece by piece (byte-balanced contiguous split, no
collective; a block of at least 1 MiB that straddles a device share is cut and its pieces' registers
are combined on the host).

tkv_crc32_batch_host_multi runs the plan with one host thread per listed device. This box has one
GPU, so device 0 stands in for each device slot ([0, 0], [0, 0, 0, 0]); the same plan, read back
through tkv_debug_multi_plan, is then run piece by piece through the device batch entry point, and
tkv_debug_multi_combine recombines those pieces: the result must equal both the multi-device call and
the oracle's CRC of every whole block. Multi-GPU scaling itself is unmeasured on hardware here (the
driver's 8-GPU SCALE run is the measurement).
"""
import numpy as np
import pytest

import tinykvpp_amd as tk
from test_multi_plan import POLY, POLY_C, combine, plan

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def mlib(lib):
    import ctypes
    VP = ctypes.c_void_p
    lib.tkv_debug_multi_plan.restype = ctypes.c_size_t
    lib.tkv_debug_multi_plan.argtypes = [ctypes.c_int, VP, VP, VP, ctypes.c_uint64, VP, ctypes.c_size_t]
    lib.tkv_debug_multi_combine.argtypes = [ctypes.c_uint32, ctypes.c_int, VP, VP, VP, ctypes.c_uint64, VP, VP]
    return lib


@pytest.mark.parametrize("ndev", [2, 4])
@pytest.mark.parametrize("algo", ["crc32", "crc32c"])
def test_plan_pieces_recombine_to_multi_device_result(gpu, oracle, mlib, ndev, algo):
    rng = np.random.default_rng(ndev * 7 + len(algo))
    # large blocks that straddle share boundaries, small ones between them, one empty block
    lens = np.array([(3 << 20) + 5, 17, 0, (5 << 20) + 123, 4096, (2 << 20) - 1, 100, (7 << 20) + 3, 59],
                    np.uint32)
    offs = np.concatenate([[3], np.cumsum(lens[:-1].astype(np.uint64) + 11) + 3]).astype(np.uint64)
    host = rng.integers(0, 256, int(offs[-1]) + int(lens[-1]) + 64, dtype=np.uint8)
    init = rng.integers(0, 1 << 32, lens.size, dtype=np.uint64).astype(np.uint32)
    got = tk.crc32_batch_host(host, offs, lens, init_raw=init, devices=[0] * ndev, algo=algo)

    rec = plan(mlib, ndev, offs, lens, init)
    assert rec[:, 0].max() == ndev - 1, "every device slot gets work"
    assert (rec[:, 5] == 0).any(), "some block is cut between devices"
    d = torch.from_numpy(host).to(gpu)
    piece_final = tk.crc32_batch(d, torch.from_numpy(rec[:, 2].astype(np.int64)).to(gpu),
                                 torch.from_numpy(rec[:, 3].astype(np.int32)).to(gpu),
                                 init_raw=torch.from_numpy(rec[:, 4].astype(np.uint32).view(np.int32)).to(gpu),
                                 algo=algo).cpu().numpy().view(np.uint32)
    recombined = combine(mlib, POLY if algo == "crc32" else POLY_C, ndev, offs, lens, init, piece_final)
    assert np.array_equal(recombined, got)
    if algo == "crc32":
        assert np.array_equal(got, oracle.batch(host, offs, lens, init))
    else:
        want = np.array([oracle.update_c(int(init[i]), host[int(offs[i]):int(offs[i]) + int(lens[i])].tobytes())
                         ^ 0xFFFFFFFF for i in range(lens.size)], np.uint32)
        assert np.array_equal(got, want)
