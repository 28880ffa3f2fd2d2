"""Multi-rank path of bench.py on CPU (gloo, world size 2): each rank checksums its own shard of the
synthetic batch (no data-path collective), and the timing/bit-exact reductions combine across
ranks. CRCs here come from the oracle; on GPUs the same decomposition runs the HIP kernel.

The second test runs bench.py's own per-rank check (verify_rank) on the real cfg2 shards
[r*1M, (r+1)*1M) of 4 KiB blocks: every block through the shard's golden XOR/SUM32 (written by
tests/golden/make_golden.py --shards from the reference crc32), and the ranks_seen count."""
import ctypes
import threading
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, q):
    import bench
    from conftest import Oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ora = Oracle(os.path.join(ROOT, "oracle", "liboracle.so"))
    first, n = bench.rank_shard(rank, 48)
    crcs = torch.from_numpy(ora.synthetic(1, first, n, 4096).view(np.int32))
    gathered = [torch.empty_like(crcs) for _ in range(world)]
    dist.all_gather(gathered, crcs)  # test-only gather to compare with the single-rank result
    elapsed, kms, ok, seen, _ = bench.reduce_timing(0.5 + rank, 1.0 + 2 * rank, rank == 0 or True, dist)
    _, _, not_ok, _, _ = bench.reduce_timing(0.1, 0.1, rank == 0, dist)
    assert seen == world
    if rank == 0:
        q.put((torch.cat(gathered).numpy().view(np.uint32), elapsed, kms, ok, not_ok))
    dist.destroy_process_group()


def test_two_rank_sharding_and_reductions(oracle):
    world, port = 2, free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, elapsed, kms, ok, not_ok = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = oracle.synthetic(1, 0, 96, 4096)
    assert np.array_equal(got, want)  # shards are disjoint, contiguous and cover the batch
    assert elapsed == pytest.approx(1.5) and kms == pytest.approx(3.0)  # max over ranks
    assert ok is True and not_ok is False  # bit_exact is the AND over ranks


def shard_crcs(ora, first, n, blen, nthreads=4):
    """Oracle CRCs of synthetic blocks [first, first + n) (fast slicing-by-8 generator path)."""
    out = np.zeros(n, np.uint32)
    fn = ora.lib.oracle_crc_synthetic_s8
    fn.argtypes = [ctypes.c_uint64] * 4 + [ctypes.c_void_p]
    step = (n + nthreads - 1) // nthreads
    ths = [threading.Thread(target=fn, args=(1, first + lo, min(n, lo + step) - lo, blen, out.ctypes.data + 4 * lo))
           for lo in range(0, n, step)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return out


def shard_worker(rank, world, port, q):
    import bench
    from conftest import Oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ora = Oracle(os.path.join(ROOT, "oracle", "liboracle.so"))
    nblocks, blen, _ = bench.CONFIGS["cfg2"]
    first, n = bench.rank_shard(rank, nblocks)
    crcs = shard_crcs(ora, first, n, blen)
    ok, full = bench.verify_rank(bench.load_oracle(), "cfg2", first, crcs, blen)
    res = bench.reduce_timing(1.0, 1.0, ok, dist, None, full)
    bad = crcs.copy()
    if rank == 1:
        bad[n // 2] ^= 1  # one wrong block deep inside rank 1's shard (past the 64-block probe)
    ok_bad, full_bad = bench.verify_rank(bench.load_oracle(), "cfg2", first, bad, blen)
    res_bad = bench.reduce_timing(1.0, 1.0, ok_bad, dist, None, full_bad)
    if rank == 0:
        q.put((res, res_bad))
    dist.destroy_process_group()


def test_two_rank_full_shard_check_and_ranks_seen():
    world, port = 2, free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res, res_bad = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    _, _, ok, seen, full = res
    assert (ok, seen, full) == (True, 2, True)  # both shards fully covered by their golden aggregates
    _, _, ok_bad, seen_bad, full_bad = res_bad
    assert (ok_bad, seen_bad, full_bad) == (False, 2, True)  # one bad block on rank 1 fails the line
