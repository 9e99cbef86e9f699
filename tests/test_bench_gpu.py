"""The bench's multi-rank path on the GPU: config 5 sharded over two ranks (torchrun, gloo for
the collectives, both ranks on the box's one GPU -- the driver's 8-GPU runs use RCCL, one rank
per GPU) must grow exactly the trees one rank grows for the same seeds: the seeds digest of the
two-rank run equals the one-rank run's.  Each run is a subprocess with its own time limit.

Two paths: `bench.py --seeds N` under torchrun, and the driver's own N > 1 command (no --seeds:
config 2 per rank plus the mandatory config-5 leg in the same world, whose `config5` object
must carry the world size and the one-rank digest)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(cmd, env):
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.timeout(600)
def test_two_ranks_shard_config5_like_one():
    env = dict(os.environ, MPT_DIST_BACKEND="gloo", MPT_BENCH_DEVICE="0")
    args = ["bench.py", "--seeds", "8", "--seed-batch", "4096", "--steps", "2", "--warmup", "2", "--no-cpu",
            "--streams", "4"]
    one = _run([sys.executable] + args, env)
    two = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args + ["--gpus", "2"], env)
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["seeds_digest"] == one["seeds_digest"]
    assert two["valid_fraction"] == one["valid_fraction"]


def _check_multi_rank_line(two, one):
    """At N > 1 the line's top level is config 2 as at N = 1 (weak scaling, one tree a rank:
    one basis for the driver's curve) and config 5 (strong scaling, seeds sharded contiguously
    over the ranks) sits under the same c5_* keys the N = 1 line carries, with the one-rank
    digest (bench.SCALING_BASIS)."""
    assert two["n_gpus"] == 2 and two["world_size"] == 2 and two["scaling"] == "weak" and two["value"] > 0
    assert two["config"]["tree_nodes"] == 20000 and two["steps"] == 3
    assert two["c5_world_size"] == 2 and two["c5_seeds"] == 12 and two["c5_value"] > 0
    assert (two["c5_steps"], two["c5_warmup"]) == (2, 3)
    assert two["c5_seeds_digest"] == one["seeds_digest"] == two["config5"]["seeds_digest"]
    assert two["config5"]["from_scratch_valid_per_s"] > 0 and two["scaling_basis"]
    assert len(json.dumps(two)) < 8000


C5_SMALL = ["--c5-seeds", "12", "--c5-steps", "2", "--c5-warmup", "3"]
C2_SMALL = ["--steps", "3", "--warmup", "1", "--tree", "20000", "--batch", "4096", "--no-cpu"]


@pytest.mark.timeout(600)
def test_driver_multi_rank_line_carries_config5():
    """`bench.py --gpus 2` as the driver launches it (under torchrun).  Sizes reduced (--tree,
    --batch, --c5-*) so the test stays short; the code path is the driver's."""
    env = dict(os.environ, MPT_DIST_BACKEND="gloo", MPT_BENCH_DEVICE="0")
    two = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2"]
               + C2_SMALL + C5_SMALL, env)
    one = _run([sys.executable, "bench.py", "--seeds", "12", "--steps", "2", "--warmup", "3", "--no-cpu"], env)
    _check_multi_rank_line(two, one)


@pytest.mark.timeout(600)
def test_gpus_flag_spawns_ranks():
    """`bench.py --gpus 2` with no torchrun around it starts the two ranks itself (a
    torch.distributed.run child, before any GPU call) and prints the same line."""
    env = dict(os.environ, MPT_DIST_BACKEND="gloo", MPT_BENCH_DEVICE="0")
    env.pop("WORLD_SIZE", None)
    two = _run([sys.executable, "bench.py", "--gpus", "2"] + C2_SMALL + C5_SMALL, env)
    one = _run([sys.executable, "bench.py", "--seeds", "12", "--steps", "2", "--warmup", "3", "--no-cpu"], env)
    _check_multi_rank_line(two, one)
