#!/usr/bin/env python3
"""Benchmark: GiB/s of CRC-32 over device-resident blocks on MI355X (BASELINE.json metric).

Workload per GPU (N=1 line = BASELINE configs[1]): 1 M x 4 KiB blocks = 4 GiB of
synthetic data (splitmix64 generator, seed 1) resident in HBM; one step = one launch of the batch
CRC kernel over the whole batch (every block checksummed, results written to HBM). With
--gpus N (torch.distributed.run, one rank per GPU) every rank checksums its own 1 M blocks
(global block ids rank*1M ...): weak scaling, no collective on the data path; the only collectives
are the timing barrier and the max-over-ranks reduction.

Prints one JSON line (rank 0). Extra fields: roofline (dominant kernel: algorithmic bytes per
launch / HIP-event launch time vs 8 TB/s HBM peak), cpu_baseline (the reference's own crc32.cpp
compiled from /root/reference into oracle/_ref, or the oracle port, on host cores over the same
buffers; plus a slicing-by-8 row that is not the reference), bit_exact (this run's CRCs vs the
oracle / golden aggregates), bit_exact_paths (post-timing parity of every other path: the one-pass
lane kernel and its fall-through, CRC-32C, device/host WAL verify on small, Zipf and adversarial images
clean and corrupted, the record check, WAL and SSTable stamps, the chained update),
pipelined_two_streams (the same steps alternating two HIP streams, as a caller checksumming a stream of
batches may run them; never `value`).
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (nblocks, block_len, description) — BASELINE.json configs; cfg4's lengths are Zipf
    "cfg2": (1 << 20, 4096, "1 M x 4 KiB WAL-record-sized blocks, device-resident"),
    "cfg3": (1 << 18, 65536, "256 K x 64 KiB SSTable data blocks, device-resident"),
    "cfg4": (1 << 17, None, "131072 blocks, Zipf sizes 256 B - 1 MiB packed back to back (unaligned), "
                            "device-resident, irregular-length path"),
    # cfg5: 4 M x 64 KiB over 8 GPUs = 512 K blocks (32 GiB) per GPU; rank r owns shard r
    "cfg5": (1 << 19, 65536, "4 M x 64 KiB sharded by batch split: 512 K x 64 KiB (32 GiB) per GPU, "
                             "device-resident"),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md


def rank_shard(rank, nblocks):
    """Weak scaling: rank r checksums global synthetic blocks [r*nblocks, (r+1)*nblocks)."""
    return rank * nblocks, nblocks


def reduce_timing(elapsed, kernel_ms, bit_exact, dist, dev=None, full=True):
    """Max over ranks of wall time and per-launch time; AND of the ranks' bit-exact checks and of
    their full-shard coverage; the number of ranks that took part (SUM of ones, must equal
    WORLD_SIZE)."""
    import torch
    t = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ok = torch.tensor([1 if bit_exact else 0, 1 if full else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    seen = torch.ones(1, dtype=torch.int32, device=dev)
    dist.all_reduce(seen, op=dist.ReduceOp.SUM)
    return float(t[0]), float(t[1]), bool(ok[0].item()), int(seen.item()), bool(ok[1].item())


def shard_golden(config, first, nblocks):
    """Golden XOR/SUM32 of synthetic blocks [first, first + nblocks) of `config` (tests/golden/
    synthetic.json "shards", written by tests/golden/make_golden.py --shards from the reference
    crc32 and the oracle), or None when no committed shard matches (then only the 64-block probe
    checks the run)."""
    with open(os.path.join(ROOT, "tests", "golden", "synthetic.json")) as f:
        g = json.load(f)
    for sh in g.get("shards", {}).get(config, []):
        if sh["first_block"] == first and sh["nblocks"] == nblocks:
            return sh
    return None


def check_shard(crcs, golden):
    """Every block of the shard against its golden aggregate (XOR and SUM32 of the CRCs)."""
    x = int(np.bitwise_xor.reduce(crcs))
    s = int(crcs.astype(np.uint64).sum() & 0xFFFFFFFF)
    return x == golden["xor"] and s == golden["sum32"]


def verify_rank(ora, config, first, crcs, blen=None, lens=None):
    """This rank's CRCs of synthetic blocks [first, first + len(crcs)): the first 64 blocks against
    the oracle, and every block against the shard's golden XOR/SUM32 when one is committed.
    Returns (bit_exact, full) where full says the whole shard was covered."""
    probe = np.zeros(64, np.uint32)
    if blen is None:
        ora.oracle_crc_synthetic_lens.argtypes = [ctypes.c_uint64] * 3 + [ctypes.c_void_p, ctypes.c_void_p]
        ora.oracle_crc_synthetic_lens(1, first, 64, np.ascontiguousarray(lens[:64], np.uint64).ctypes.data,
                                      probe.ctypes.data)
    else:
        ora.oracle_crc_synthetic(1, first, 64, blen, probe.ctypes.data)
    ok = bool(np.array_equal(crcs[:64], probe))
    gold = shard_golden(config, first, crcs.size)
    if gold is not None:
        ok = ok and check_shard(crcs, gold)
    return ok, gold is not None


def warm_up(step, steps, min_ms):
    """At least `steps` untimed steps, continued until `min_ms` of wall time have passed: the
    shader clock ramps over the first few hundred ms of load, and a handful of steps (--warmup 5 is
    ~4 ms on cfg2) leaves the timed steps on a cold clock (profiles/r1/irr_compare_warmup.txt: the
    first rounds read up to 10 % low). Steps are issued in groups of 8 with a sync between groups,
    so the host does not queue seconds of work ahead of the clock check."""
    import torch
    t0 = time.perf_counter()
    done = 0
    while done < steps or (time.perf_counter() - t0) * 1e3 < min_ms:
        for _ in range(8 if done >= steps else min(8, steps - done)):
            step()
            done += 1
        torch.cuda.synchronize()
    return done, (time.perf_counter() - t0) * 1e3


def pmc_traffic(csv_path, config):
    """HBM read bytes of one step from a rocprofv3 --pmc FETCH_SIZE pass of this bench command (a
    separate run: counters are never collected inside the timed run): per kernel of the step, the
    median over its dispatches, summed. FETCH_SIZE is in KiB and counts half the bytes of a wide
    streaming read on gfx950, so bytes = FETCH_SIZE*1024*2 (MI355X_MICROARCH.md §HBM). Default
    source: the committed profile of this config, newest round first (profiles/r6/final/ holds cfg2-cfg5
    on the round-6 tree, tools/gpu_evidence.sh)."""
    import csv
    from collections import defaultdict
    step_kernels = (("crc_rows", "crc_stream", "rows_tile_scan", "rows_scan_tiles",
                     "rows_finish", "crc_fixup") if config == "cfg4" else ("crc_packed",))
    path = csv_path
    if path is None:
        for cand in (os.path.join(ROOT, "profiles", "r6", "final", f"pmc_{config}_FETCH_SIZE.csv"),
                     os.path.join(ROOT, "profiles", "r5", "final", f"pmc_{config}_FETCH_SIZE.csv"),
                     os.path.join(ROOT, "profiles", "r4", "final", f"pmc_{config}_FETCH_SIZE.csv"),
                     os.path.join(ROOT, "profiles", "r3", "pmc", f"pmc_{config}_FETCH_SIZE.csv"),
                     os.path.join(ROOT, "profiles", "r2", f"pmc_{config}", "FETCH_SIZE_counters.csv"),
                     os.path.join(ROOT, "profiles", "r1", f"pmc_{config}", "p3_counters.csv")):
            if os.path.exists(cand):
                path = cand
                break
    if path is None or not os.path.exists(path):
        return None, None
    per = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != "FETCH_SIZE":
            continue
        name = r.get("Kernel_Name", "")
        for k in step_kernels:
            if k in name:
                per[k].append(float(r["Counter_Value"]))
    if not per:
        return None, None
    kib = sum(float(np.median(v)) for v in per.values())
    return round(kib * 1024 * 2), os.path.relpath(path, ROOT) + " (FETCH_SIZE x 1024 x 2, summed over the step's kernels)"


def load_oracle():
    o = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
    o.oracle_crc_synthetic.argtypes = [ctypes.c_uint64] * 4 + [ctypes.c_void_p]
    return o


def cpu_baseline(host, nblocks, blen, seconds_target=16.0, total_blocks=None, offs=None, lens=None):
    """Time the reference crc32 (oracle/_ref, else the oracle port) on host cores over a bounded
    contiguous sample of the batch's own bytes; contiguous per-thread block ranges. Uniform blocks
    of `blen` bytes, or (offs, lens) for an irregular batch (blen = mean length, for the sizing)."""
    ref_path = os.path.join(ROOT, "oracle", "_ref", "libref_crc32.so")
    if offs is None:
        offs = np.arange(nblocks, dtype=np.uint64) * blen
        lens = np.full(nblocks, blen, np.uint32)
    offs = np.ascontiguousarray(offs, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint32)
    if os.path.exists(ref_path):
        lib = ctypes.CDLL(ref_path)
        fn = lib.ref_crc32_irregular
        fn.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_size_t, ctypes.c_void_p]
        kind = "reference"
    else:
        lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
        lib.oracle_crc_batch.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint64, ctypes.c_void_p]
        fn = None
        kind = "port"

    def run(lo, hi, out):
        if fn is not None:
            fn(host.ctypes.data, offs.ctypes.data + lo * 8, lens.ctypes.data + lo * 4, hi - lo, out.ctypes.data + lo * 4)
        else:
            lib.oracle_crc_batch(host.ctypes.data, offs.ctypes.data + lo * 8, lens.ctypes.data + lo * 4, None, hi - lo,
                                 out.ctypes.data + lo * 4)

    cores = max(1, min(len(os.sched_getaffinity(0)), 16))  # the GPU box's CPU share is 16
    out = np.zeros(nblocks, np.uint32)
    # calibrate on 1 thread; the sample is at most the batch (the bytes already copied to the host)
    t0 = time.perf_counter()
    cal = min(nblocks, 4096)
    run(0, cal, out)
    per_block = (time.perf_counter() - t0) / cal
    one_core_gibs = int(lens[:cal].astype(np.uint64).sum()) / (1 << 30) / max(per_block * cal, 1e-9)
    sample = int(min(nblocks, max(cores * 1024, seconds_target * cores / max(per_block, 1e-12))))
    step = (sample + cores - 1) // cores
    ranges = [(min(sample, i * step), min(sample, (i + 1) * step)) for i in range(cores)]  # contiguous, maybe empty
    # passes over the sample until ~seconds_target core-seconds of CRC work have run (>= 1 pass)
    passes, dt = 0, 0.0
    while passes == 0 or (dt * cores < seconds_target and passes < 8):
        ths = [threading.Thread(target=run, args=(lo, hi, out)) for lo, hi in ranges]
        t0 = time.perf_counter()
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        dt += time.perf_counter() - t0
        passes += 1
    sbytes = int(lens[:sample].astype(np.uint64).sum())
    # SURVEY §8d's optional comparison row, NOT the reference algorithm: slicing-by-8 on the same
    # sample, threads and ranges (oracle/crc32_oracle.c), one pass.
    s8lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
    s8 = s8lib.oracle_crc_batch_s8
    s8.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_void_p]
    out8 = np.zeros(sample, np.uint32)
    s8lib.oracle_update_s8(ctypes.c_uint32(0), None, ctypes.c_size_t(0))  # build its tables before the threads

    def run8(lo, hi):
        s8(host.ctypes.data, offs.ctypes.data + lo * 8, lens.ctypes.data + lo * 4, hi - lo, out8.ctypes.data + lo * 4)

    ths = [threading.Thread(target=run8, args=(lo, hi)) for lo, hi in ranges]
    t8 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    t8 = time.perf_counter() - t8
    slicing8 = {"value": round(sbytes / (1 << 30) / t8, 4), "unit": "GiB/s", "cores": cores,
                "kind": "not reference: slicing-by-8 (oracle/crc32_oracle.c), same sample and threads, one pass",
                "agrees_with_reference": bool(np.array_equal(out8, out[:sample]))}
    what = f"{blen} B blocks" if lens.min() == lens.max() else "blocks (Zipf lengths)"
    return {"value": round(passes * sbytes / (1 << 30) / dt, 4), "unit": "GiB/s", "cores": cores, "kind": kind,
            "sample": f"{passes} pass(es) over the first {sample} of the {total_blocks or nblocks} {what}, "
                      f"{sbytes / (1 << 30):.2f} GiB (same bytes as the GPU run), {cores} threads, contiguous block "
                      f"ranges, {dt:.2f} s wall, ~{dt * cores:.0f} core-seconds",
            "one_core_gibs": round(one_core_gibs, 4), "slicing_by_8": slicing8}, out[:sample]


def prepare(cfg, first, nblocks, dev, ora):
    """Synthetic batch of `cfg` (rank shard [first, first + nblocks)) resident in HBM, and one step
    over it: (step(stream, out), bytes per step, blen, lens, offs, data)."""
    import torch
    import tinykvpp_amd as tk
    _, blen, _ = CONFIGS[cfg]
    if blen is None:  # cfg4: Zipf lengths computed on the host, packed, unaligned
        lens = np.zeros(nblocks, np.uint64)
        ora.oracle_zipf_lengths.argtypes = [ctypes.c_uint64] * 3 + [ctypes.c_void_p]
        ora.oracle_zipf_lengths(1, first, nblocks, lens.ctypes.data)
        offs = np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.int64)
        total = int(lens.sum())
        data = torch.empty(total + 64, dtype=torch.uint8, device=dev)
        d_off = torch.from_numpy(offs).to(dev)
        d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
        tk.fill_synthetic_blocks(data, d_off, d_len, first_block=first)

        def step(strm, o):
            tk.crc32_batch(data, d_off, d_len, out=o, stream=strm)
        keep = (d_off, d_len)
    else:
        lens, offs, keep = None, None, ()
        total = nblocks * blen
        data = torch.empty(total, dtype=torch.uint8, device=dev)
        tk.fill_synthetic_uniform(data, blen, nblocks, first_block=first)

        def step(strm, o):
            tk.crc32_batch_uniform(data, blen, nblocks, out=o, stream=strm)
    torch.cuda.synchronize()
    return {"step": step, "total": total, "blen": blen, "lens": lens, "offs": offs, "data": data, "keep": keep}


def time_steps(step, out, stream, steps, barrier=None):
    """K back-to-back steps on one stream between one HIP event pair, bracketed by barrier() (ranks)
    and a device sync on both sides: (wall s, device ms per step)."""
    import torch
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if barrier is not None:
        barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        step(stream, out)
    ev1.record(stream)
    torch.cuda.synchronize()
    if barrier is not None:
        barrier()
    return time.perf_counter() - t0, ev0.elapsed_time(ev1) / steps


def roofline(total, kernel_ms, cfg, traffic_csv=None):
    traffic, traffic_src = pmc_traffic(traffic_csv, cfg)
    achieved = total / (kernel_ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
            "kernel_ms": round(kernel_ms, 4), "algorithmic_bytes_per_launch": total}


def host_legs(cfg_ctx, crcs):
    """cfg3 "+ H2D/D2H timed" (BASELINE configs[2]): the same blocks starting and ending in pinned host
    memory, through tkv_crc32_batch_host, two ways: staged (hipMemcpyAsync of 256 MiB slabs to HBM on
    two streams, the kernel there, results back) and zero-copy (the kernels read the pinned buffer in
    place over PCIe). Never `value`."""
    import torch
    import tinykvpp_amd as tk
    lib = tk.load_library()
    total, blen = cfg_ctx["total"], cfg_ctx["blen"]
    nblocks = total // blen
    host_p = torch.empty(total, dtype=torch.uint8).pin_memory()
    host_p.copy_(cfg_ctx["data"])
    hp = host_p.numpy()
    offs_h = np.arange(nblocks, dtype=np.uint64) * blen
    lens_h = np.full(nblocks, blen, np.uint32)
    legs = {}
    for name, mapped in (("staged_hipMemcpyAsync", 0), ("zero_copy", 1)):
        prev = lib.tkv_debug_set_host_mapped(mapped)
        try:
            got = tk.crc32_batch_host(hp, offs_h, lens_h)
            t0 = time.perf_counter()
            for _ in range(2):
                tk.crc32_batch_host(hp, offs_h, lens_h)
            dt = (time.perf_counter() - t0) / 2
        finally:
            lib.tkv_debug_set_host_mapped(prev)
        legs[name] = {"value": round(total / (1 << 30) / dt, 2), "unit": "GiB/s", "GB_per_s": round(total / 1e9 / dt, 2),
                      "bit_exact": bool(np.array_equal(got, crcs))}
    legs["source"] = "pinned host memory in, host results out, whole batch per call, mean of 2 calls after one untimed"
    del host_p, hp
    return legs


def bit_exact_paths(dev, ora, quick=False):
    """Post-timing parity checks of the paths the headline batch never reaches,
    each against the oracle (oracle/liboracle.so: Sarwate CRC, the sequential WAL decode of
    wal.cpp:63-130, the WAL stamp of wal.cpp:54-58, the SSTable stamp) on seeded synthetic inputs:
      list_lanes_one_pass   >= 1 M gapped 26-59 B WAL payloads through tkv_crc32_batch_device (the
                            one-pass crc_list_lanes kernel; tkv_debug_irregular_path 0)
      list_pack_one_pass    the same batch with one 65 B block near its end (the wave that meets it
                            switches to crc_list_lanes' packed mode: path 1)
      list_lanes_fall_through  the same batch with one 1025 B block (the general path: path 2)
      crc32c_list_lanes     the one-pass batch under CRC-32C (sampled against the oracle)
      wal_verify_device_*   tkv_wal_verify_device on small-record, Zipf and values-made-of-records
                            images, clean and with one flipped payload byte: same (status, records
                            decoded, stop offset) as the sequential decode
      wal_verify_host       tkv_wal_verify (host image, copied to HBM), clean and corrupted
      wal_check_records     tkv_wal_check_records_device (record starts known), clean and corrupted
      wal_stamp             tkv_wal_stamp (group commit) byte-identical to the oracle's stamps
      sst_stamp             tkv_sst_stamp_blocks vs oracle_sst_stamp; verify finds one flipped byte
      update_chain          tkv_crc32_update_device chained over odd spans of a device buffer
    Nothing here is inside a timed region. quick: smaller inputs (smoke())."""
    import torch
    import tinykvpp_amd as tk
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import wal_images
    wo = wal_images.load(os.path.join(ROOT, "oracle", "liboracle.so"))
    lib = tk.load_library()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ora.oracle_crc_batch.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint64, ctypes.c_void_p]
    ora.oracle_update_c.restype = ctypes.c_uint32
    ora.oracle_update_c.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
    ora.oracle_sst_stamp.restype = ctypes.c_uint32
    ora.oracle_sst_stamp.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    ora.oracle_crc32.restype = ctypes.c_uint32
    ora.oracle_crc32.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    res = {}
    rng = np.random.default_rng(2026)

    def u32(t):
        return t.cpu().numpy().view(np.uint32)

    # ---- irregular batches of WAL-payload-sized blocks -------------------------------------------
    nb = 1_100_003  # (>= 1 M blocks: the one-pass kernel's threshold)
    lens = rng.integers(26, 60, nb).astype(np.int64)
    offs = 3 + 8 + np.concatenate([[0], np.cumsum(lens[:-1] + 8)])  # an 8-byte record prefix before each
    host = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    for name, tweak, want_path in (("list_lanes_one_pass", None, 0), ("list_pack_one_pass", (nb - 5, 65), 1),
                                   ("list_lanes_fall_through", (nb - 40, 1025), 2)):
        ln = lens.copy()
        if tweak is not None:
            ln[tweak[0]] = tweak[1]
        o, l32 = torch.from_numpy(offs).to(dev), torch.from_numpy(ln.astype(np.int32)).to(dev)
        got = u32(tk.crc32_batch(d, o, l32))
        kp = lib.tkv_debug_irregular_path(st)
        ph = lib.tkv_debug_irregular_phases(st)
        want = np.zeros(nb, np.uint32)
        o64, l32h = offs.astype(np.uint64), ln.astype(np.uint32)  # (named: alive across the call)
        ora.oracle_crc_batch(host.ctypes.data, o64.ctypes.data, l32h.ctypes.data, None, nb, want.ctypes.data)
        path_ok = kp == want_path and (ph == 0) == (want_path != 2)
        res[name] = {"ok": bool(np.array_equal(got, want)) and path_ok, "blocks": nb, "mismatches":
                     int((got != want).sum()), "kernel_path": int(kp), "general_path_phases": int(ph),
                     "path_as_expected": path_ok}
        if tweak is None:
            gc = u32(tk.crc32_batch(d, o, l32, algo="crc32c"))
            smp = rng.choice(nb, 4000 if quick else 20000, replace=False)
            wc = np.array([ora.oracle_update_c(0xFFFFFFFF, host.ctypes.data + int(offs[i]), int(ln[i])) ^ 0xFFFFFFFF
                           for i in smp], np.uint32)
            res["crc32c_list_lanes"] = {"ok": bool(np.array_equal(gc[smp], wc)), "sampled": int(smp.size)}
    del d

    # ---- WAL recovery verify on the device ---------------------------------------------------------
    sizes = {"small": 150_000 if quick else 1_500_000, "zipf": 10_000 if quick else 100_000,
             "values_of_records": 6_000 if quick else 60_000}
    U64 = ctypes.c_uint64
    for shape, n in sizes.items():
        img, roffs, rsize = wal_images.image(wo, shape, n, seed=len(shape))
        want_clean = wal_images.decode(wo, img)
        entry = {"records": n, "bytes": int(img.size), "oracle_clean": list(want_clean)}
        ok = want_clean == ("ok", n, img.size)
        dimg = torch.from_numpy(img).to(dev)
        bad = n - 777
        flip = int(roffs[bad] + rsize[bad] - 1)  # the record's last payload byte
        for tag in ("clean", "corrupted"):
            if tag == "corrupted":
                img[flip] ^= 0x01
                dimg[flip] ^= 0x01
            want = wal_images.decode(wo, img)
            if tag == "corrupted":
                ok = ok and want == ("corrupted", bad, int(roffs[bad]))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            got = tk.wal.verify_device(dimg)
            ms = (time.perf_counter() - t0) * 1e3
            rounds = (U64 * 4)()
            lib.tkv_debug_wal_last(rounds)
            entry[tag] = {"device": list(got), "oracle": list(want), "ms": round(ms, 3), "device_rounds": rounds[0]}
            ok = ok and tuple(got) == want
            if shape == "small":  # the host-image entry point and the record check on the same image
                hv = tk.wal.verify(img)
                res.setdefault("wal_verify_host", {"ok": True})
                res["wal_verify_host"][tag] = list(hv)
                res["wal_verify_host"]["ok"] &= tuple(hv) == want
                ro = torch.from_numpy(roffs.astype(np.int32)).to(dev)
                fb, crc = tk.wal.check_records_device(dimg, ro)
                fbv = int(fb.item())
                stored = img[(roffs + 4)[:, None].astype(np.int64) + np.arange(4)].copy().view("<u4").ravel()
                want_fb = bad if tag == "corrupted" else n
                crc_ok = bool(np.array_equal(np.delete(u32(crc), bad), np.delete(stored, bad)))
                res.setdefault("wal_check_records", {"ok": True})
                res["wal_check_records"][tag] = {"first_bad": fbv, "want": want_fb}
                res["wal_check_records"]["ok"] &= fbv == want_fb and crc_ok
        entry["ok"] = bool(ok)
        res[f"wal_verify_device_{shape}"] = entry
        if shape == "small":  # group-commit stamp of the same records, against the oracle's bytes
            img[flip] ^= 0x01
            m = min(n, 200_000)
            end = int(roffs[m - 1] + rsize[m - 1])
            un = img[:end].copy()
            for b in range(4, 8):
                un[roffs[:m].astype(np.int64) + b] = 0
            sz32 = rsize[:m].astype(np.uint32)
            check_rc = lib.tkv_wal_stamp(ctypes.c_void_p(un.ctypes.data), ctypes.c_void_p(roffs.ctypes.data),
                                         ctypes.c_void_p(sz32.ctypes.data), ctypes.c_uint64(m))
            res["wal_stamp"] = {"ok": check_rc == 0 and bool(np.array_equal(un, img[:end])), "records": m}
        del dimg, img

    # ---- SSTable data-block stamps ------------------------------------------------------------------
    nimg = 2000
    isz = rng.integers(22, 9000, nimg).astype(np.uint64)
    ioff = np.concatenate([[0], np.cumsum(isz[:-1])]).astype(np.uint64)
    f = rng.integers(0, 256, int(isz.sum()), dtype=np.uint8)
    tk.sst.stamp_blocks(f, ioff, isz)
    stamped = f[(ioff + 17)[:, None].astype(np.int64) + np.arange(4)].copy().view("<u4").ravel()
    want = np.array([ora.oracle_sst_stamp(f.ctypes.data + int(o), int(s)) for o, s in zip(ioff, isz)], np.uint32)
    v_ok = tk.sst.verify_blocks(f, ioff, isz) == ("ok", 0, nimg)
    f[int(ioff[1234] + isz[1234] // 2)] ^= 0x10
    v_bad = tk.sst.verify_blocks(f, ioff, isz)
    res["sst_stamp"] = {"ok": bool(np.array_equal(stamped, want)) and v_ok and v_bad == ("corrupted", 1, 1234),
                        "images": nimg, "verify_corrupted": list(v_bad)}

    # ---- the drop-in update, chained over device spans ---------------------------------------------
    buf = rng.integers(0, 256, 5_000_003, dtype=np.uint8)
    dbuf = torch.from_numpy(buf).to(dev)
    cuts = np.sort(rng.choice(buf.size, 9, replace=False))
    c = tk.crc32()
    prev = 0
    for cut in list(cuts) + [buf.size]:
        c.update(dbuf[prev:cut])
        prev = int(cut)
    res["update_chain"] = {"ok": c.finalize() == ora.oracle_crc32(buf.ctypes.data, buf.size), "spans": int(cuts.size + 1)}
    torch.cuda.synchronize()
    for k in res:
        res[k]["ok"] = bool(res[k]["ok"])
    res["all_ok"] = all(v["ok"] for v in res.values())
    return res


def wal_payload_batches(dev, ora, quick=False):
    """Irregular batches of WAL payloads through tkv_crc32_batch_device (the reference's records are
    record_len = 18 + |k| + |v| bytes, wal.cpp:25, each payload 8 header bytes after the previous one,
    wal.cpp:54-58): the one-pass kernel's lane and packed modes. 1 GiB of payload
    per batch (32 MiB with quick) in a random device buffer, 5 untimed then 20 timed launches between
    one event pair on the launch stream; GB/s of payload; which path folded the batch
    (tkv_debug_irregular_path: 0 lanes, 1 packed); 20 000 sampled blocks against the oracle. Never
    `value`."""
    import torch
    import tinykvpp_amd as tk
    lib = tk.load_library()
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    ora.oracle_crc_batch.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint64, ctypes.c_void_p]
    rng = np.random.default_rng(2606)
    target = (32 << 20) if quick else (1 << 30)
    data = torch.randint(0, 256, (target * 2 + 4096,), dtype=torch.uint8, device=dev)
    host = data.cpu().numpy()
    wal = np.array([26, 28, 33, 36, 59])
    shapes = (("36 B", 36, lambda n: np.full(n, 36)),
              ("26-59 B", 36, lambda n: rng.choice(wal, n)),
              ("26-59 B + 2 % of 65-400 B", 40,
               lambda n: np.where(rng.random(n) < 0.02, rng.integers(65, 401, n), rng.choice(wal, n))),
              ("65-256 B", 160, lambda n: rng.integers(65, 257, n)),
              ("180-400 B", 290, lambda n: rng.integers(180, 401, n)),
              ("300-1000 B", 650, lambda n: rng.integers(300, 1001, n)))
    res = {"source": "8-byte gaps (WAL headers), 5 untimed + 20 timed launches, GB/s of payload"}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, mean, draw in shapes:
        n = target // (mean + 8)
        lens = draw(n).astype(np.int64)
        offs = 8 + np.concatenate([[0], np.cumsum(lens[:-1] + 8)])
        o = torch.from_numpy(offs).to(dev)
        ln = torch.from_numpy(lens.astype(np.int32)).to(dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        args = (ctypes.c_void_p(data.data_ptr()), ctypes.c_void_p(o.data_ptr()), ctypes.c_void_p(ln.data_ptr()), None,
                ctypes.c_void_p(out.data_ptr()), n, sp)
        for _ in range(5):
            assert lib.tkv_crc32_batch_device(*args) == 0
        e0.record(st)
        for _ in range(20):
            lib.tkv_crc32_batch_device(*args)
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        kp = lib.tkv_debug_irregular_path(sp)
        got = out.cpu().numpy().view(np.uint32)
        smp = np.sort(rng.choice(n, min(n, 20_000), replace=False))
        so, sl = offs[smp].astype(np.uint64), lens[smp].astype(np.uint32)
        want = np.zeros(smp.size, np.uint32)
        ora.oracle_crc_batch(host.ctypes.data, so.ctypes.data, sl.ctypes.data, None, smp.size, want.ctypes.data)
        res[name] = {"blocks": int(n), "payload_bytes": int(lens.sum()), "ms": round(ms, 4),
                     "GB_per_s": round(int(lens.sum()) / ms / 1e6, 1), "kernel_path": int(kp),
                     "bit_exact_sampled": bool(np.array_equal(got[smp], want))}
        del o, ln, out
    del data
    torch.cuda.empty_cache()
    return res


def build_identity():
    """The build id baked into the loaded library against the hash of this tree's sources."""
    from tinykvpp_amd import build_id
    try:
        lib_id, tree, same = build_id.check()
    except AttributeError:  # a library built before tkv_build_id existed
        lib_id, tree, same = None, build_id.source_hash(), False
    if not same:
        print(f"bench.py: WARNING: libtkv_crc32.so build id {lib_id} != tree source hash {tree}", file=sys.stderr)
    return {"library": lib_id, "tree": tree, "match": same}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--min-warmup-ms", type=float, default=1000.0,
                    help="keep warming up (untimed) until this much wall time has passed (clock ramp)")
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="cfg3: skip the host-memory end-to-end measurement")
    ap.add_argument("--no-pipelined", action="store_true", help="skip the two-stream pipelined rate (extra field)")
    ap.add_argument("--no-more-configs", action="store_true",
                    help="cfg2: skip timing cfg3, cfg4 and cfg5 (N=1) or cfg5 (N>1) in the same run (more_configs)")
    ap.add_argument("--no-paths", action="store_true",
                    help="skip the post-timing parity checks of the other paths (bit_exact_paths)")
    ap.add_argument("--no-wal-payloads", action="store_true",
                    help="skip the irregular WAL-payload batches (wal_payload_batches; N=1 only)")
    ap.add_argument("--traffic-csv", default=None,
                    help="rocprofv3 --pmc counter_collection.csv (FETCH_SIZE) of this command, for roofline.traffic")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import tinykvpp_amd as tk

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # One rank per GPU. TKV_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share devices
    # round-robin); the default, nccl (RCCL), carries only the barrier and the timing max-reduce.
    backend = os.environ.get("TKV_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    tk.set_device(local)
    dev = torch.device("cuda", local)
    # TKV_BENCH_FORCE_DIST=1 runs the process group, barriers and reductions even at WORLD_SIZE 1
    # (under torch.distributed.run), so a one-GPU box exercises the multi-rank code path over RCCL.
    use_dist = world > 1 or os.environ.get("TKV_BENCH_FORCE_DIST") == "1"
    if use_dist:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    nblocks, blen, desc = CONFIGS[args.config]
    first, nblocks = rank_shard(rank, nblocks)
    ora = load_oracle()
    stream = torch.cuda.current_stream()
    out = torch.empty(nblocks, dtype=torch.int32, device=dev)
    ctx = prepare(args.config, first, nblocks, dev, ora)
    step, total, lens, offs, data = ctx["step"], ctx["total"], ctx["lens"], ctx["offs"], ctx["data"]

    if use_dist:
        # The first collective builds the communicator (RCCL: hundreds of ms). Paid here, before the
        # warm-up, so the barrier in front of the timed steps is short and the clocks stay up: with
        # the lazy build there, the timed steps of a one-rank RCCL run read 7 % low
        # (profiles/r2/dist/bench_nccl_ws1_lazy.json).
        dist.barrier()
        reduce_timing(0.0, 0.0, True, dist, dev if backend == "nccl" else None)
    warm_steps, warm_ms = warm_up(lambda: step(None, out), args.warmup, args.min_warmup_ms)

    # One HIP event pair on the launch stream brackets the K steps; the average launch duration is
    # their span / K. Event markers between steps would each hold the next launch back by ~10 us
    # (rocprofv3 kernel trace: back-to-back launches start 0 us after their predecessor ends,
    # 10.4 us with two markers between them), a cost no caller pays.
    elapsed, kernel_ms = time_steps(step, out, stream, args.steps, dist.barrier if use_dist else None)

    # correctness of this exact buffer, from the last timed step (checked after the timed region so
    # no CPU pause lets the clocks fall between warmup and timing)
    crcs = out.cpu().numpy().view(np.uint32).copy()
    bit_exact, full = verify_rank(ora, args.config, first, crcs, blen, None if blen else lens)
    ranks_seen = 1
    if use_dist:
        elapsed, kernel_ms, bit_exact, ranks_seen, full = reduce_timing(
            elapsed, kernel_ms, bit_exact, dist, dev if backend == "nccl" else None, full)
    if full:
        scope = f"every block of every rank's shard (golden XOR/SUM32 of blocks [r*{nblocks}, (r+1)*{nblocks})) " \
                "and its first 64 blocks against the oracle"
    else:
        scope = "first 64 blocks of each rank's shard against the oracle (no committed golden aggregate for some shard)"

    bytes_per_step = total
    total_bytes = bytes_per_step * args.steps * world
    value = total_bytes / (1 << 30) / elapsed

    line = {
        "metric": "GiB/s CRC32 over device-resident blocks (4 KiB & 64 KiB) on 1 MI355X",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "warmup_run": {"steps": warm_steps, "ms": round(warm_ms, 1), "min_ms": args.min_warmup_ms,
                       "note": "untimed; at least --warmup steps, continued until min_ms of wall time (clock ramp)"},
        "ms_per_step": round(elapsed * 1e3 / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (SURVEY §8d splitmix64 generator, seed 1), generated in HBM",
        "config": {"workload": f"{args.config}: {desc}", "blocks_per_gpu": nblocks, "block_bytes": blen or "zipf",
                   "bytes_per_gpu_per_step": bytes_per_step, "parallelism": f"batch split x{world}, no collective"},
        "bit_exact": bit_exact,
        "bit_exact_scope": scope,
        "ranks_seen": ranks_seen,
        "roofline": roofline(bytes_per_step, kernel_ms, args.config, args.traffic_csv),
        "cpu_baseline": None,
        "build": build_identity(),
    }
    if world == 1 and not args.no_pipelined:
        # A caller checksumming a stream of batches may alternate two HIP streams: each launch's
        # workgroups then take the CUs its predecessor's tail frees. Same K steps,
        # same work per step, results checked; reported beside `value`, never as `value`.
        strms = [torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)]
        outs = [out, torch.empty_like(out)]
        for i in range(20):
            step(strms[i % 2], outs[i % 2])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(strms[i % 2], outs[i % 2])
        torch.cuda.synchronize()
        dt2 = time.perf_counter() - t0
        same = bool(torch.equal(outs[0], outs[1])) and bool(np.array_equal(outs[0].cpu().numpy().view(np.uint32), crcs))
        line["pipelined_two_streams"] = {"value": round(total * args.steps / (1 << 30) / dt2, 2), "unit": "GiB/s",
                                         "ms_per_step": round(dt2 * 1e3 / args.steps, 4), "bit_exact": same,
                                         "note": "consecutive steps alternate two streams; not `value`"}
        del outs, strms
    if args.config == "cfg3" and not args.no_e2e:
        line["e2e_host"] = host_legs(ctx, crcs)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if blen is not None:
            nb_host = min(nblocks, (4 << 30) // blen)  # at most 4 GiB of the batch goes to host memory
            host = data[:nb_host * blen].cpu().numpy()
            cb, cpu_crcs = cpu_baseline(host, nb_host, blen, total_blocks=nblocks)
        else:  # cfg4: the leading blocks up to 4 GiB, at their own (unaligned) offsets
            nb_host = int(np.searchsorted(offs + lens.astype(np.int64), 4 << 30, side="right"))
            host = data[:int(offs[nb_host - 1] + lens[nb_host - 1])].cpu().numpy()
            cb, cpu_crcs = cpu_baseline(host, nb_host, max(1, int(lens[:nb_host].mean())), total_blocks=nblocks,
                                        offs=offs[:nb_host], lens=lens[:nb_host])
        cb["agrees_with_gpu"] = bool(np.array_equal(cpu_crcs, crcs[:cpu_crcs.size]))
        line["cpu_baseline"] = cb
        del host
    if args.config == "cfg2" and not args.no_more_configs:
        # The metric's other half (64 KiB blocks, cfg3, with its host legs), the irregular path (cfg4) and
        # the 8-GPU shard config (cfg5: each rank its own 512 K x 64 KiB shard, rank r = global blocks
        # [r * 512 K, (r + 1) * 512 K)), timed in this same run exactly as the main line is: warm-up with
        # the clock floor, K steps between one event pair (bracketed by barriers across ranks), every
        # block checked against the golden aggregates. At N > 1 only cfg5 runs (the scaling config), its
        # aggregate = all ranks' bytes / the max over ranks of the wall time. Never `value`.
        del ctx, step, data, out
        torch.cuda.empty_cache()
        more = {}
        for cfg in (("cfg3", "cfg4", "cfg5") if world == 1 else ("cfg5",)):
            nb, bl, dsc = CONFIGS[cfg]
            f0, nb = rank_shard(rank, nb) if cfg == "cfg5" else (0, nb)
            c = prepare(cfg, f0, nb, dev, ora)
            o = torch.empty(nb, dtype=torch.int32, device=dev)
            if use_dist:
                dist.barrier()
            warm_up(lambda: c["step"](None, o), args.warmup, args.min_warmup_ms)
            el, kms = time_steps(c["step"], o, stream, args.steps, dist.barrier if use_dist else None)
            cr = o.cpu().numpy().view(np.uint32).copy()
            ok, fl = verify_rank(ora, cfg, f0, cr, bl, None if bl else c["lens"])
            seen = 1
            if use_dist:
                el, kms, ok, seen, fl = reduce_timing(el, kms, ok, dist, dev if backend == "nccl" else None, fl)
            entry = {"workload": f"{cfg}: {dsc}", "value": round(c["total"] * args.steps * world / (1 << 30) / el, 2),
                     "unit": "GiB/s", "n_gpus": world, "ms_per_step": round(el * 1e3 / args.steps, 4),
                     "roofline": roofline(c["total"], kms, cfg), "bit_exact": ok, "ranks_seen": seen,
                     "bit_exact_scope": ("every block of every rank's shard (golden XOR/SUM32) and the first 64 "
                                         "against the oracle") if fl else "first 64 blocks against the oracle"}
            if cfg == "cfg5":
                entry["shards"] = f"rank r: global blocks [r*{nb}, (r+1)*{nb}); value = {world} shards' bytes / max wall"
            if cfg == "cfg3" and not args.no_e2e:
                entry["e2e_host"] = host_legs(c, cr)
            more[cfg] = entry
            del c, o
            torch.cuda.empty_cache()
        line["more_configs"] = more
    if world == 1 and args.config == "cfg2" and not args.no_wal_payloads:
        torch.cuda.empty_cache()
        line["wal_payload_batches"] = wal_payload_batches(dev, ora)
    if not args.no_paths:
        # after every timed region: parity of the paths the timed batches never reach (every rank checks
        # on its own GPU; the line carries rank 0's details and the AND over ranks)
        torch.cuda.empty_cache()
        paths = bit_exact_paths(dev, ora)
        if use_dist:
            ok = torch.tensor([1 if paths["all_ok"] else 0], dtype=torch.int32,
                              device=dev if backend == "nccl" else None)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            paths["all_ranks_ok"] = bool(ok.item())
        line["bit_exact_paths"] = paths
    if rank == 0:
        print(json.dumps(line), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
