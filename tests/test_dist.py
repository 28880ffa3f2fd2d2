"""Multi-rank path of bench.py on CPU (gloo, world size 2): each rank checksums its own shard of the
synthetic batch (no data-path collective), and the timing/bit-exact reductions combine across
ranks. CRCs here come from the oracle; on GPUs the same decomposition runs the HIP kernel."""
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
    elapsed, kms, ok = bench.reduce_timing(0.5 + rank, 1.0 + 2 * rank, rank == 0 or True, dist)
    _, _, not_ok = bench.reduce_timing(0.1, 0.1, rank == 0, dist)
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
