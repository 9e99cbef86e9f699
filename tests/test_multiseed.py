"""CPU: the multi-GPU path (independent seeds, one collective at the end) with a world of two
gloo ranks.  Each rank grows the trees of its shard of seeds with the oracle's batched
round (the same round the device engine runs, tests/test_engine_gpu.py); the per-seed tree
digests gathered from both ranks must equal the digests of one process running every seed,
and the reduced counters must be the sums."""
import os
import socket
import sys
import time

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from motionplanningtoolkit_amd import multiseed, scenes

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))

N_SEEDS, N0, K, ROUNDS = 6, 400, 96, 3


def grow(seed):
    """Oracle rounds for one seed: tree digest and valid count."""
    import oracle as orc

    sc = scenes.omni_scenario()
    rng = np.random.default_rng(seed)
    nodes = np.zeros((N0 + ROUNDS * K, sc.dim))
    nodes[:N0] = rng.uniform(sc.ranges[:, 0], sc.ranges[:, 1], size=(N0, sc.dim))
    par = np.zeros(nodes.shape[0], np.int32)
    bvh = orc.BVH(sc.env_tris)
    n = N0
    for r in range(ROUNDS):
        n, _, _ = orc.engine_step(sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, seed, r * K, K, bvh, sc.env_tf,
                                  sc.agent_tris, nodes, par, n)
    return multiseed.tree_digest(nodes[:n], par[:n]), n - N0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t0 = time.perf_counter()
        digests, valid = {}, 0
        for i in multiseed.shard_seeds(N_SEEDS, world, rank):
            seed = multiseed.rank_seed(1000, i)
            digests[seed], v = grow(seed)
            valid += v
        elapsed, (valid_sum, n_trees) = multiseed.reduce_run(dist, time.perf_counter() - t0,
                                                             [valid, len(digests)], "cpu")
        allg = multiseed.gather_digests(dist, digests)
        if rank == 0:
            np.save(os.path.join(out_dir, "result.npy"),
                    np.array([repr(sorted(allg.items())), valid_sum, n_trees, elapsed], dtype=object),
                    allow_pickle=True)
    finally:
        dist.destroy_process_group()


def test_shard_seeds_partition():
    for n, w in ((256, 8), (10, 3), (3, 4), (0, 2)):
        seen = [i for r in range(w) for i in multiseed.shard_seeds(n, w, r)]
        assert seen == list(range(n))
    assert list(multiseed.shard_seeds(256, 8, 1)) == list(range(32, 64))


def test_reduce_run_single_process():
    assert multiseed.reduce_run(None, 1.5, [3, 4], "cpu") == (1.5, [3, 4])
    assert multiseed.gather_digests(None, {1: "a"}) == {1: "a"}


@pytest.mark.timeout(300)
def test_two_rank_gloo_matches_one_process(tmp_path):
    mp.spawn(_rank_main, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    res = np.load(os.path.join(tmp_path, "result.npy"), allow_pickle=True)  # written by this test
    gathered, valid_sum, n_trees = res[0], int(res[1]), int(res[2])
    single = {}
    total = 0
    for i in range(N_SEEDS):
        seed = multiseed.rank_seed(1000, i)
        single[seed], v = grow(seed)
        total += v
    assert gathered == repr(sorted(single.items()))
    assert valid_sum == total and n_trees == N_SEEDS
    assert len(set(single.values())) == N_SEEDS  # seeds give different trees
