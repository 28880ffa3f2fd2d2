#!/usr/bin/env python3
"""Stream-mode probe (not product code): back-to-back batches of 64 B - 20 KiB blocks through several
builds of libtkv_crc32.so, each checked block by block against the oracle; prints the first wrong
blocks with their row and segment lane. Run on the GPU box (reads GRAFT_REPO_ROOT)."""
import ctypes, os, sys
import numpy as np, torch
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"]); sys.path.insert(0, os.path.join(os.environ["GRAFT_REPO_ROOT"], "tests"))
from conftest import Oracle
VP,U64=ctypes.c_void_p,ctypes.c_uint64
torch.cuda.set_device(0)
ora=Oracle(os.path.join(os.environ["GRAFT_REPO_ROOT"],"oracle","liboracle.so"))
libs=[]
for p in sys.argv[1:]:
    l=ctypes.CDLL(os.path.abspath(p)); l.tkv_crc32_batch_device.argtypes=[VP,VP,VP,VP,VP,U64,VP]; assert l.tkv_set_device(0)==0; libs.append(l)
rng=np.random.default_rng(1)
for case in range(4):
    lens=rng.integers(64, [200,600,3000,20000][case], 3000).astype(np.int64)
    start=int(rng.integers(0,16))
    offs=(start+np.concatenate([[0],np.cumsum(lens[:-1])])).astype(np.int64)
    host=rng.integers(0,256,int(offs[-1]+lens[-1])+64,dtype=np.uint8)
    d=torch.from_numpy(host).cuda(); o=torch.from_numpy(offs).cuda(); ln=torch.from_numpy(lens.astype(np.int32)).cuda()
    want=ora.batch(host,offs,lens)
    st=VP(torch.cuda.current_stream().cuda_stream)
    for p,l in zip(sys.argv[1:],libs):
        out=torch.zeros(len(lens),dtype=torch.int32,device="cuda")
        assert l.tkv_crc32_batch_device(VP(d.data_ptr()),VP(o.data_ptr()),VP(ln.data_ptr()),None,VP(out.data_ptr()),len(lens),st)==0
        torch.cuda.synchronize()
        got=out.cpu().numpy().view(np.uint32)
        bad=np.flatnonzero(got!=want)
        info=[]
        for bb in bad[:6]:
            e=int(offs[bb]+lens[bb])-(start - (start & 15)) ; info.append((int(bb), int(lens[bb]), e//4096, (e%4096+63)//64-1))
        print(case, os.path.basename(p), "bad", bad.size, info, flush=True)
