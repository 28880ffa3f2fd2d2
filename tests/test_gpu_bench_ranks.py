"""bench.py's multi-rank code path on the one GPU of a test box, launched the way the driver launches
the scaling runs (python -m torch.distributed.run ... bench.py --gpus N):

* one rank over RCCL with TKV_BENCH_FORCE_DIST=1: the process group, the barriers around the timed
  steps and the max/min/sum reductions run on the device, as on an 8-GPU node;
* two ranks sharing the GPU over gloo (TKV_BENCH_BACKEND=gloo): rank 1 checksums global blocks
  [1 M, 2 M), which only its committed golden shard aggregate can check, and ranks_seen must be 2.

Each line must report every block of every rank's shard bit-exact against tests/golden/synthetic.json
(written from the reference's own crc32.cpp by tests/golden/make_golden.py)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_bench(nproc, extra_env, config="cfg2", more=False):
    env = dict(os.environ, **extra_env)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(nproc), "--config", config, "--steps", "3", "--warmup", "1", "--min-warmup-ms", "0",
           "--no-cpu-baseline", "--no-pipelined", "--no-e2e"] + ([] if more else ["--no-more-configs"])
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints the one line
    return json.loads(lines[0])


@pytest.mark.gpu
def test_bench_one_rank_over_rccl(gpu):
    line = run_bench(1, {"TKV_BENCH_FORCE_DIST": "1"}, more=True)
    for cfg in ("cfg3", "cfg4", "cfg5"):
        m = line["more_configs"][cfg]
        assert m["bit_exact"] is True and m["ranks_seen"] == 1, (cfg, m)
        assert m["bit_exact_scope"].startswith("every block"), (cfg, m)
    assert line["n_gpus"] == 1 and line["ranks_seen"] == 1
    assert line["bit_exact"] is True
    assert line["bit_exact_scope"].startswith("every block of every rank's shard")
    # the WAL-payload batches: lane mode for lane blocks only, the packed mode once longer values appear
    w = line["wal_payload_batches"]
    for name, want in (("36 B", 0), ("26-59 B", 0), ("26-59 B + 2 % of 65-400 B", 1), ("65-256 B", 1),
                       ("180-400 B", 1), ("300-1000 B", 1)):
        assert w[name]["bit_exact_sampled"] is True and w[name]["kernel_path"] == want, (name, w[name])


@pytest.mark.gpu
def test_bench_two_ranks_cfg5_leg(gpu):
    """The multi-rank line carries the cfg5 leg: each rank checksums its own 32 GiB shard
    of BASELINE configs[4] (rank 1 = global blocks [512 K, 1 M), checked only by its committed golden
    shard aggregate), and the leg's aggregate is both shards' bytes over the max wall time."""
    line = run_bench(2, {"TKV_BENCH_BACKEND": "gloo"}, "cfg2", more=True)
    assert set(line["more_configs"]) == {"cfg5"}
    m = line["more_configs"]["cfg5"]
    assert m["n_gpus"] == 2 and m["ranks_seen"] == 2
    assert m["bit_exact"] is True
    assert m["bit_exact_scope"].startswith("every block of every rank's shard")
    assert m["value"] > 0 and m["ms_per_step"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["cfg2", "cfg4"])
def test_bench_two_ranks_share_the_gpu(gpu, config):
    line = run_bench(2, {"TKV_BENCH_BACKEND": "gloo"}, config)
    assert line["n_gpus"] == 2 and line["ranks_seen"] == 2
    assert line["bit_exact"] is True
    assert line["bit_exact_scope"].startswith("every block of every rank's shard")
