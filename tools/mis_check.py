# correctness of unaligned dwordx4 loads: run the misaligned probes with FIN=2 (per-row XOR of the row's
# dwords read at base+MIS) and compare with a host computation
import ctypes, os, sys, numpy as np, torch
ROOT = os.getcwd(); sys.path.insert(0, ROOT)
import tinykvpp_amd as tk
lib = ctypes.CDLL("tools/libexplore.so"); lib.explore_name.restype = ctypes.c_char_p
lib.explore_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
names = [lib.explore_name(i).decode() for i in range(lib.explore_count())]
torch.cuda.set_device(0); tk.set_device(0)
n = 4096 * 8
host = np.random.default_rng(0).integers(0, 256, n * 4096 + 64, dtype=np.uint8)
d = torch.from_numpy(host).cuda()
for mis in (0, 4, 5, 8):
    i = names.index(f"pat seg64 D4 fin2 mis{mis}")
    out = torch.zeros(n, dtype=torch.int32, device="cuda")
    assert lib.explore_run(i, ctypes.c_void_p(d.data_ptr()), n, 4096, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)[: n - 1]
    rows = host[mis: mis + (n - 1) * 4096].reshape(n - 1, 4096).view(np.uint32)
    want = np.bitwise_xor.reduce(rows, axis=1)
    print(mis, "OK" if np.array_equal(got, want) else f"MISMATCH {np.sum(got != want)}")
