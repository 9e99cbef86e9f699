"""Multi-GPU runs over independent seeds.

A single RRT tree does not shard: every extension depends on the previous insertions
(planners/rrt.hpp:44-86).  Multi-GPU work is therefore independent trees: rank r of W owns
its own seeds, builds its own tree, and nothing crosses ranks on the data path.  The one
collective is the end-of-run reduction of timings (max) and counters (sum), plus an
allgather of per-seed digests so a run on W GPUs can be checked against the same seeds on
one GPU.  The counter-based RNG of the engine (fcl_math.h engine_uniform) keys every draw by
(seed, extension index), so a seed's tree does not depend on which rank grows it.
"""
from __future__ import annotations

import hashlib

import numpy as np


def rank_seed(seed_base: int, rank: int) -> int:
    """bench.py: one tree per rank."""
    return seed_base + rank


def shard_seeds(n_seeds: int, world: int, rank: int) -> range:
    """Seeds [0, n_seeds) in contiguous blocks: seed i runs on rank floor(i / ceil(n/world))
    (256 seeds, 32 per GPU on 8 GPUs)."""
    per = -(-n_seeds // world)
    return range(min(rank * per, n_seeds), min((rank + 1) * per, n_seeds))


def tree_digest(states: np.ndarray, parents: np.ndarray) -> str:
    """Bitwise digest of a tree (state bytes + parent ids)."""
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(states, np.float64).tobytes())
    h.update(np.ascontiguousarray(parents, np.int32).tobytes())
    return h.hexdigest()


def reduce_run(dist, elapsed: float, counters: list, device) -> tuple:
    """Max of the ranks' elapsed times and sums of their counters (the bench's only
    collective; RCCL on GPUs, gloo in the CPU tests)."""
    import torch

    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return elapsed, [int(c) for c in counters]
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    s = torch.tensor([float(c) for c in counters], dtype=torch.float64, device=device)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    return float(t.item()), [int(v) for v in s.tolist()]


def gather_digests(dist, digests: dict) -> dict:
    """Union of every rank's {seed: digest}."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return dict(digests)
    parts = [None] * dist.get_world_size()
    dist.all_gather_object(parts, digests)
    out = {}
    for p in parts:
        out.update(p)
    return out
