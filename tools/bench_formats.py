#!/usr/bin/env python3
"""Throughput of the SURVEY §8f rows on one MI355X (one JSON line each):

  wal_stamp    group commit: tkv_wal_stamp over N encoded records in host memory (wal.cpp:54-58)
  wal_verify   recovery: tkv_wal_verify over the slurped WAL image (wal.cpp:63-130, engine.cpp:31-53):
               image copied to HBM, chain walk + CRC batch on the device; also for an image already
               in HBM (tkv_wal_verify_device) and for a 1 GiB WAL of 26-90 B records
  sst_stamp    tkv_sst_stamp_blocks over a host SSTable image of ~4 KiB data blocks
  sst_device   tkv_sst_block_crcs_device over the same images resident in HBM (kernel + fix-up)
  crc32c_cfg2  CRC-32C over 1 M x 4 KiB device-resident blocks (cfg2 shape)
  uniform_512B, uniform_64B  the same 4 GiB as 8 M x 512 B and 64 M x 64 B blocks (crc_packed_small)

Host-memory rows include the PCIe copies (pageable source: host memcpy into pinned staging). Beside
each row, "cpu_reference" times the reference's own path on one host core over the same bytes: its
crc32.cpp compiled into oracle/_ref, driven by oracle/ref_shim.cpp's restatement of wal_entry::decode's
loop (recovery), encode's stamp (group commit), or one crc32 per block (SSTable), with the results
checked against the GPU's. The reference is single-threaded on these paths.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import tinykvpp_amd as tk  # noqa: E402
import tinykvpp_amd.sst as sst  # noqa: E402
from conftest import Oracle  # noqa: E402

torch.cuda.set_device(0)
tk.set_device(0)
lib = tk.load_library()
ora = Oracle(os.path.join(ROOT, "oracle", "liboracle.so"))
ref = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libref_crc32.so"))
ref.ref_wal_verify.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
ref.ref_wal_stamp.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
ref.ref_crc32_irregular.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]


def cpu_ref(nbytes, secs, agrees, what):
    return {"cpu_reference": {"GB/s": round(nbytes / secs / 1e9, 3), "ms": round(secs * 1e3, 1), "cores": 1,
                              "kind": "reference", "what": what, "agrees_with_gpu": bool(agrees)}}


def ref_wal_verify(img):
    g, p = ctypes.c_uint64(), ctypes.c_uint64()
    t0 = time.perf_counter()
    rc = ref.ref_wal_verify(ctypes.c_void_p(img.ctypes.data), img.size, ctypes.byref(g), ctypes.byref(p))
    return time.perf_counter() - t0, ("ok" if rc == 0 else "corrupted", g.value, p.value)
rng = np.random.default_rng(1)
GiB = 1 << 30


def emit(name, nbytes, secs, unit_count, extra=None):
    line = {"row": name, "GB/s": round(nbytes / secs / 1e9, 2), "bytes": int(nbytes), "units": int(unit_count),
            "ms": round(secs * 1e3, 3)}
    line.update(extra or {})
    print(json.dumps(line), flush=True)


def timeit(fn, reps=5):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


# ---- WAL image: records with Zipf-ish key/value sizes (wal.cpp:19-61 layout) -------------------------
n_rec = 400_000
klen = rng.integers(8, 64, n_rec).astype(np.uint32)
vlen = np.minimum(rng.zipf(1.6, n_rec) * 64, 16_000).astype(np.uint32)
size = 26 + klen + vlen
offs = np.concatenate([[0], np.cumsum(size[:-1], dtype=np.uint64)]).astype(np.uint64)
total = int(size.sum())
wal = rng.integers(0, 256, total, dtype=np.uint8)
hdr = np.zeros((n_rec, 26), np.uint8)
hdr[:, 0:4] = (size - 8).astype("<u4").view(np.uint8).reshape(-1, 4)
hdr[:, 8] = 0
hdr[:, 9:17] = np.arange(n_rec, dtype="<u8").view(np.uint8).reshape(-1, 8)
hdr[:, 17] = 0
hdr[:, 18:22] = klen.astype("<u4").view(np.uint8).reshape(-1, 4)
hdr[:, 22:26] = vlen.astype("<u4").view(np.uint8).reshape(-1, 4)
idx = offs.astype(np.int64)[:, None] + np.arange(26)
wal[idx] = hdr
sizes32 = size.astype(np.uint32)


def stamp():
    tk.check(lib.tkv_wal_stamp(ctypes.c_void_p(wal.ctypes.data), ctypes.c_void_p(offs.ctypes.data),
                               ctypes.c_void_p(sizes32.ctypes.data), n_rec))


t = timeit(stamp)
# the reference's encode stamp over the same records, on a copy (wal.cpp:54-58), one core
wal_ref = wal.copy()
t0 = time.perf_counter()
ref.ref_wal_stamp(ctypes.c_void_p(wal_ref.ctypes.data), ctypes.c_void_p(offs.ctypes.data),
                  ctypes.c_void_p(sizes32.ctypes.data), n_rec)
cpu = time.perf_counter() - t0
emit("wal_stamp", total, t, n_rec, {"records": n_rec, **cpu_ref(total, cpu, np.array_equal(wal_ref, wal),
                                                                 "wal_entry::encode's stamp per record")})
del wal_ref

good, stop = ctypes.c_uint64(), ctypes.c_uint64()


def verify():
    rc = lib.tkv_wal_verify(ctypes.c_void_p(wal.ctypes.data), total, ctypes.byref(good), ctypes.byref(stop))
    assert rc == 0 and good.value == n_rec and stop.value == total, (rc, good.value, stop.value)


t = timeit(verify)
cpu, res = ref_wal_verify(wal)
emit("wal_verify", total, t, n_rec, {"records": n_rec, "verified": good.value,
                                     **cpu_ref(total, cpu, res == ("ok", good.value, stop.value),
                                               "wal_entry::decode until the image ends")})
poffs, plens = offs + 8, (size - 8).astype(np.uint32)
t = timeit(lambda: tk.crc32_batch_host(wal, poffs, plens))
emit("wal_payload_batch_host", total, t, n_rec, {"what": "the CRC part of wal_verify alone"})
t0 = time.perf_counter()
for _ in range(3):
    lib.tkv_wal_verify(ctypes.c_void_p(wal.ctypes.data), total, ctypes.byref(good), ctypes.byref(stop))
t1 = time.perf_counter()
for _ in range(3):
    stamp()
t2 = time.perf_counter()
emit("wal_verify_vs_stamp_back_to_back", total, (t1 - t0) / 3, n_rec, {"stamp_ms": round((t2 - t1) / 3 * 1e3, 3)})

# same WAL image in pinned host memory (a WAL append buffer allocated with hipHostMalloc): the kernels
# read it in place, no staging copies
wal_pin_t = torch.from_numpy(wal).pin_memory()
wal_pin = wal_pin_t.numpy()
t = timeit(lambda: tk.check(lib.tkv_wal_stamp(ctypes.c_void_p(wal_pin.ctypes.data), ctypes.c_void_p(offs.ctypes.data),
                                              ctypes.c_void_p(sizes32.ctypes.data), n_rec)))
emit("wal_stamp_pinned", total, t, n_rec, {"records": n_rec, "source": "pinned, read in place"})


def verify_pinned():
    rc = lib.tkv_wal_verify(ctypes.c_void_p(wal_pin.ctypes.data), total, ctypes.byref(good), ctypes.byref(stop))
    assert rc == 0 and good.value == n_rec and stop.value == total, (rc, good.value, stop.value)


t = timeit(verify_pinned)
emit("wal_verify_pinned", total, t, n_rec, {"records": n_rec, "verified": good.value, "source": "pinned, read in place"})
t = timeit(lambda: tk.crc32_batch_host(wal_pin, poffs, plens))
emit("wal_payload_batch_host_pinned", total, t, n_rec, {"what": "the CRC part of wal_verify_pinned alone"})
del wal_pin, wal_pin_t

# the same image already resident in HBM (tkv_wal_verify_device: walk + CRC batch + first-bad search)
wal_dev = torch.from_numpy(wal).cuda()
t = timeit(lambda: tk.wal.verify_device(wal_dev))
assert tk.wal.verify_device(wal_dev) == ("ok", n_rec, total)
emit("wal_verify_device", total, t, n_rec, {"records": n_rec, "source": "device-resident image"})
del wal_dev

# ---- WAL of small records (26-90 B: puts of short keys and values), 1 GiB: the walk dominates -----------
sk = rng.integers(4, 24, 20_000_000).astype(np.uint32)
sv = rng.integers(0, 40, 20_000_000).astype(np.uint32)
ssz = 26 + sk + sv
n_small = int(np.searchsorted(np.cumsum(ssz, dtype=np.uint64), np.uint64(1 << 30)))
sk, sv, ssz = sk[:n_small], sv[:n_small], ssz[:n_small]
soffs_w = np.concatenate([[0], np.cumsum(ssz[:-1], dtype=np.uint64)]).astype(np.uint64)
stotal = int(ssz.sum())
swal = rng.integers(0, 256, stotal, dtype=np.uint8)
for col, vals in ((0, ssz - 8), (18, sk), (22, sv)):
    for b in range(4):
        swal[soffs_w.astype(np.int64) + col + b] = ((vals >> (8 * b)) & 0xFF).astype(np.uint8)
for col in (8, 17):
    swal[soffs_w.astype(np.int64) + col] = 0
ssz32 = ssz.astype(np.uint32)
tk.check(lib.tkv_wal_stamp(ctypes.c_void_p(swal.ctypes.data), ctypes.c_void_p(soffs_w.ctypes.data),
                           ctypes.c_void_p(ssz32.ctypes.data), n_small))
assert tk.wal.verify(swal) == ("ok", n_small, stotal)
t = timeit(lambda: tk.wal.verify(swal), reps=3)
cpu, res = ref_wal_verify(swal)
emit("wal_verify_small_records", stotal, t, n_small, {"records": n_small, "mean_record_bytes": round(stotal / n_small, 1),
                                                     "source": "pageable host image",
                                                     **cpu_ref(stotal, cpu, res == ("ok", n_small, stotal),
                                                               "wal_entry::decode until the image ends")})
swal_pin_t = torch.from_numpy(swal).pin_memory()
t = timeit(lambda: tk.wal.verify(swal_pin_t.numpy()), reps=3)
emit("wal_verify_small_records_pinned", stotal, t, n_small, {"records": n_small, "source": "pinned host image"})
del swal_pin_t
swal_dev = torch.from_numpy(swal).cuda()
assert tk.wal.verify_device(swal_dev) == ("ok", n_small, stotal)
t = timeit(lambda: tk.wal.verify_device(swal_dev))
emit("wal_verify_small_records_device", stotal, t, n_small, {"records": n_small, "source": "device-resident image"})
# the previous design: record_len chain walked on host threads, CRCs in one GPU batch
host_walk = []
for k in range(1):
    t0 = time.perf_counter()
    cnt = lib.tkv_debug_wal_chain(ctypes.c_void_p(swal.ctypes.data), stotal, None, 0, None, None)
    host_walk.append(time.perf_counter() - t0)
emit("wal_small_records_host_chain_walk_only", stotal, float(np.median(host_walk)), int(cnt),
     {"what": "tkv_debug_wal_chain: the host-thread walk alone (the exact fallback)"})
del swal_dev, swal

# ---- SSTable image: ~4 KiB data blocks -----------------------------------------------------------------
nblk = 250_000
body = 4096 - 36
sizes = np.full(nblk, 36 + body, np.uint64)
soffs = (np.arange(nblk, dtype=np.uint64) * sizes[0]).astype(np.uint64)
sfile = rng.integers(0, 256, int(sizes.sum()), dtype=np.uint8)
sfile[soffs.astype(np.int64)] = 20


def sstamp():
    sst.stamp_blocks(sfile, soffs, sizes)


t = timeit(sstamp)
# the reference's crc32 over each stamped block image with its field read as zero: on a copy with
# the fields zeroed, one core (the reference never computes these fields; parity unpinned)
zf = sfile.copy()
zf[soffs.astype(np.int64)[:, None] + np.arange(17, 21)] = 0
rcrc = np.zeros(nblk, np.uint32)
sz32 = sizes.astype(np.uint32)
t0 = time.perf_counter()
ref.ref_crc32_irregular(ctypes.c_void_p(zf.ctypes.data), ctypes.c_void_p(soffs.ctypes.data),
                        ctypes.c_void_p(sz32.ctypes.data), nblk, ctypes.c_void_p(rcrc.ctypes.data))
cpu = time.perf_counter() - t0
stamped = sfile[soffs.astype(np.int64)[:, None] + np.arange(17, 21)].copy().view("<u4").ravel()
emit("sst_stamp", sfile.nbytes, t, nblk, {"block_image_bytes": int(sizes[0]),
                                          **cpu_ref(sfile.nbytes, cpu, np.array_equal(rcrc, stamped),
                                                    "crc32 per block image, field as zero")})
del zf
assert sst.verify_blocks(sfile, soffs, sizes)[0] == "ok"
sfile_pin_t = torch.from_numpy(sfile).pin_memory()
sfile_pin = sfile_pin_t.numpy()
t = timeit(lambda: sst.stamp_blocks(sfile_pin, soffs, sizes))
emit("sst_stamp_pinned", sfile.nbytes, t, nblk, {"block_image_bytes": int(sizes[0]), "source": "pinned, read in place"})
t = timeit(lambda: sst.verify_blocks(sfile_pin, soffs, sizes))
emit("sst_verify_pinned", sfile.nbytes, t, nblk, {"block_image_bytes": int(sizes[0]), "source": "pinned, read in place"})
assert np.array_equal(sfile_pin, sfile)
del sfile_pin, sfile_pin_t

d = torch.from_numpy(sfile).cuda()
do = torch.from_numpy(soffs.astype(np.int64)).cuda()
ds = torch.from_numpy(sizes.astype(np.int32)).cuda()
out = torch.empty(nblk, dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream()
for _ in range(20):
    sst.block_crcs_device(d, do, ds, out=out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(st)
for _ in range(50):
    sst.block_crcs_device(d, do, ds, out=out)
e1.record(st)
torch.cuda.synchronize()
t = e0.elapsed_time(e1) / 50 / 1e3
want = sfile[soffs.astype(np.int64)[:, None] + np.arange(17, 21)].copy().view("<u4").ravel()
emit("sst_device", sfile.nbytes, t, nblk, {"bit_exact_vs_host_stamp": bool(np.array_equal(out.cpu().numpy().view(np.uint32), want))})
del d

# ---- CRC-32C, cfg2 shape ---------------------------------------------------------------------------------
n = 1 << 20
data = torch.empty(n * 4096, dtype=torch.uint8, device="cuda")
tk.fill_synthetic_uniform(data, 4096, n)
outc = torch.empty(n, dtype=torch.int32, device="cuda")
for _ in range(100):
    tk.crc32_batch_uniform(data, 4096, n, out=outc, algo="crc32c")
e0.record(st)
for _ in range(100):
    tk.crc32_batch_uniform(data, 4096, n, out=outc, algo="crc32c")
e1.record(st)
torch.cuda.synchronize()
t = e0.elapsed_time(e1) / 100 / 1e3
probe = data[:64 * 4096].cpu().numpy()
ok = all(ora.crc_c(probe[i * 4096:(i + 1) * 4096].tobytes()) == int(outc[i:i + 1].cpu().numpy().view(np.uint32)[0])
         for i in range(0, 64, 7))
emit("crc32c_cfg2", n * 4096, t, n, {"frac_of_8TB/s": round(n * 4096 / t / 8e12, 4), "bit_exact_sample": ok})

# ---- small uniform blocks (sector-sized checksums, crc_packed_small) --------------------
for blen in (512, 64):
    nb = (n * 4096) // blen
    outs = torch.empty(nb, dtype=torch.int32, device="cuda")
    for _ in range(20):
        tk.crc32_batch_uniform(data, blen, nb, out=outs)
    e0.record(st)
    for _ in range(50):
        tk.crc32_batch_uniform(data, blen, nb, out=outs)
    e1.record(st)
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 50 / 1e3
    ok = all(ora.crc(probe[i * blen:(i + 1) * blen].tobytes()) == int(outs[i:i + 1].cpu().numpy().view(np.uint32)[0])
             for i in range(0, 64 * 4096 // blen, 7))
    emit(f"uniform_{blen}B", nb * blen, t, nb, {"frac_of_8TB/s": round(nb * blen / t / 8e12, 4),
                                               "bit_exact_sample": ok})

# ---- latency of small calls (the per-record drop-in path and small group commits) ----------------------
def lat(fn, reps=200):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps * 1e6


res = ctypes.c_uint32()
for nbytes in (36, 4096, 65536, 262144, 1 << 20, 16 << 20):
    payload = rng.integers(0, 256, nbytes, dtype=np.uint8)
    us = lat(lambda: tk.check(lib.tkv_crc32_update(0xFFFFFFFF, ctypes.c_void_p(payload.ctypes.data), nbytes,
                                                   ctypes.byref(res))), reps=50)
    ok = (res.value ^ 0xFFFFFFFF) == ora.crc(payload.tobytes())
    print(json.dumps({"row": "update_latency", "bytes": nbytes, "us_per_call": round(us, 2), "bit_exact": ok}),
          flush=True)
for nrec in (1, 16, 256, 4096):
    recs = np.ascontiguousarray(wal[:int(offs[nrec])]) if nrec < n_rec else wal
    o = offs[:nrec].copy()
    s32 = sizes32[:nrec].copy()
    us = lat(lambda: tk.check(lib.tkv_wal_stamp(ctypes.c_void_p(recs.ctypes.data), ctypes.c_void_p(o.ctypes.data),
                                               ctypes.c_void_p(s32.ctypes.data), nrec)), reps=50)
    print(json.dumps({"row": "wal_stamp_latency", "records": nrec, "bytes": int(offs[nrec]), "us_per_call": round(us, 2)}),
          flush=True)
