import ctypes, numpy as np, torch, sys, os
VP, U64 = ctypes.c_void_p, ctypes.c_uint64
torch.cuda.set_device(0)
lib = ctypes.CDLL(os.path.abspath(sys.argv[1]))
lib.tkv_crc32_batch_device.argtypes = [VP, VP, VP, VP, VP, U64, VP]
lib.tkv_debug_irregular_lists.argtypes = [VP, VP]
assert lib.tkv_set_device(0) == 0
d = torch.zeros(1 << 30, dtype=torch.uint8, device='cuda')
st = VP(torch.cuda.current_stream().cuda_stream)
for blen, gap in ((128, 8), (36, 8), (64, 0)):
    n = (1 << 30) // (blen + gap) - 1
    offs = torch.arange(n, dtype=torch.int64, device='cuda') * (blen + gap)
    lens = torch.full((n,), blen, dtype=torch.int32, device='cuda')
    out = torch.empty(n, dtype=torch.int32, device='cuda')
    for r in range(3):
        s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
        s.record()
        assert lib.tkv_crc32_batch_device(VP(d.data_ptr()), VP(offs.data_ptr()), VP(lens.data_ptr()), None, VP(out.data_ptr()), n, st) == 0
        e.record(); torch.cuda.synchronize()
        o = (ctypes.c_uint32 * 3)()
        lib.tkv_debug_irregular_lists(st, o)
        print(blen, gap, n, "ms", round(s.elapsed_time(e), 3), "quit_waves", o[0], "loop_iters", o[1], "waves", o[2], flush=True)
