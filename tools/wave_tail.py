#!/usr/bin/env python3
"""Per-wave start/end times of the packed kernel (s_memrealtime, 100 MHz): how long the slowest
waves keep the launch alive after the median wave has finished (tail of a static partition)."""
import ctypes, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tinykvpp_amd as tk
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libexplore.so"))
lib.explore_stamped.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
torch.cuda.set_device(0); tk.set_device(0)
DYN = int(sys.argv[1]) if len(sys.argv) > 1 else 0  # 1: dynamically scheduled packed body
n = 1 << 20
data = torch.empty(n * 4096, dtype=torch.uint8, device="cuda")
tk.fill_synthetic_uniform(data, 4096, n)
out = torch.empty(n, dtype=torch.int32, device="cuda")
ref = tk.crc32_batch_uniform(data, 4096, n).clone()
W = torch.cuda.get_device_properties(0).multi_processor_count * 16
st = torch.empty(2 * W, dtype=torch.int64, device="cuda")
sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
wg_ends = []
for rep in range(4):
    assert lib.explore_stamped(ctypes.c_void_p(data.data_ptr()), n, ctypes.c_void_p(out.data_ptr()),
                               ctypes.c_void_p(st.data_ptr()), sp, DYN) == 0
    torch.cuda.synchronize()
    assert torch.equal(out, ref), "stamped kernel output differs"
    s = st.cpu().numpy().reshape(-1, 2).astype(np.float64) * 10.0  # ns
    t0 = s[:, 0].min()
    start, end = s[:, 0] - t0, s[:, 1] - t0
    dur = end - start
    wg_ends.append(end.reshape(-1, 16).max(axis=1))
    print(f"rep {rep}: kernel span {end.max()/1e3:.1f} us; wave end p50 {np.median(end)/1e3:.1f} "
          f"p90 {np.percentile(end, 90)/1e3:.1f} p99 {np.percentile(end, 99)/1e3:.1f} max {end.max()/1e3:.1f} us; "
          f"start spread {start.max()/1e3:.1f} us; dur p50 {np.median(dur)/1e3:.1f} min {dur.min()/1e3:.1f} max {dur.max()/1e3:.1f}",
          flush=True)
# per-XCD view (blocks round-robin over 8 XCDs: wave w -> WG w//16 -> XCD (w//16) % 8, a label only)
xcd = (np.arange(W) // 16) % 8
for x in range(8):
    print(f"xcd-group {x}: median wave duration {np.median(dur[xcd == x])/1e3:.1f} us, max end {end[xcd == x].max()/1e3:.1f}")
# per wave slot inside the workgroup (0..15): is the spread systematic (issue arbitration) or random?
slot = np.arange(W) % 16
print("median wave duration by slot (us): " + " ".join(f"{np.median(dur[slot == k])/1e3:.0f}" for k in range(16)))
wg = np.arange(W) // 16
wgdur = np.array([end[wg == g].max() for g in range(W // 16)])
print(f"workgroup end (slowest wave) p10/p50/p90/max: {np.percentile(wgdur,10)/1e3:.0f}/{np.median(wgdur)/1e3:.0f}/"
      f"{np.percentile(wgdur,90)/1e3:.0f}/{wgdur.max()/1e3:.0f} us")
rank = np.argsort(np.argsort(dur.reshape(-1, 16), axis=1), axis=1)  # 0 = fastest wave of its workgroup
print("mean rank (0 = fastest in its workgroup) by slot: " + " ".join(f"{rank[:, k].mean():.1f}" for k in range(16)))
# is a workgroup's lateness systematic (same blockIdx late in every launch) or random?
E = np.array(wg_ends)
E = E - E.mean(axis=1, keepdims=True)
c = np.corrcoef(E)
print("correlation of workgroup end times between launches: " +
      " ".join(f"{c[i, j]:.2f}" for i in range(len(E)) for j in range(i + 1, len(E))))
