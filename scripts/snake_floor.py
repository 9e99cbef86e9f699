"""Config 3's NN against the floor of any index that prunes on x, y.

The snake's state is (x, y, speeds, 11 link angles): the grid index prunes cells on x, y only,
so every tree node whose x, y partial distance to the query is below the query's final best
squared distance must be examined by any such index (its full distance cannot be ruled out
from x, y alone).  This script runs the bench's config-3 round (100 k-node tree, K = 65 536,
the same seed), reads the engine's examined-point counter, and counts that floor per query
on the GPU (torch, exact float64 partial distances).  Prints one JSON line.

  python scripts/snake_floor.py [--tree 100000] [--batch 65536] [--seed 1000]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tree", type=int, default=100_000)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--seed", type=int, default=1000)
    ap.add_argument("--chunk", type=int, default=512)
    ap.add_argument("--ppc", type=float, default=0.0, help="grid points per cell (0: the engine's default)")
    a = ap.parse_args()

    import torch

    import motionplanningtoolkit_amd as mpt
    from motionplanningtoolkit_amd import multiseed, scenes

    mpt.init(0)
    sc = scenes.snake_scenario("corridor")
    seed = multiseed.rank_seed(a.seed, 0)
    rng = np.random.default_rng(seed)
    n0, K = a.tree, a.batch
    tree = rng.uniform(sc.ranges[:, 0], sc.ranges[:, 1], size=(n0, sc.dim))
    env = mpt.Environment(sc.env_tris, sc.env_tf)
    agent = mpt.AgentMesh(sc.agent_tris)
    eng = mpt.RRTEngine(env, agent, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, n0 + K, seed)
    eng.add_nodes(tree)
    eng.set_nn("auto", a.ppc)
    eng.enable_timing(True)
    stream = torch.cuda.current_stream()
    for _ in range(3):  # the bench's warm-up rounds
        eng.set_size(n0, stream)
        eng.step(K, stream)
    eng.set_size(n0, stream)
    eng.collide_stats(True)
    eng.step(K, stream)
    torch.cuda.synchronize()
    st = eng.collide_stats(False)
    times = eng.kernel_times()
    samples, nn, _, _ = eng.last_round(K)
    nodes, _ = eng.read_tree(n0)
    eng.close()

    dev = torch.device("cuda", 0)
    T = torch.from_numpy(nodes).to(dev)
    Q = torch.from_numpy(samples).to(dev)
    ids = torch.from_numpy(nn.astype(np.int64)).to(dev) - 1  # 1-based node ids
    best = ((Q - T[ids]) ** 2).sum(1)  # FLANN's squared L2 of each query's answer
    floor = torch.zeros(K, dtype=torch.int64, device=dev)
    txy = T[:, :2]
    for c in range(0, K, a.chunk):
        q = Q[c:c + a.chunk, :2]
        pxy = ((q[:, None, :] - txy[None, :, :]) ** 2).sum(2)  # x, y partial squared distances
        floor[c:c + a.chunk] = (pxy < best[c:c + a.chunk, None]).sum(1)
    # a spot check that the answers are the nearest (the parity tests cover this in full)
    sub = torch.arange(0, K, max(1, K // 128), device=dev)
    d_all = ((Q[sub, None, :] - T[None, :, :]) ** 2).sum(2)
    spot_ok = bool((d_all.min(1).values == best[sub]).all().item())

    examined = st["nn_points"] / K
    fl = floor.double().mean().item()
    out = {
        "metric": "config-3 NN points examined per query vs the x, y index floor",
        "config": {"workload": "snake_trailers (11 links) in the corridor", "tree": n0, "queries": K, "seed": seed,
                   "ppc": a.ppc},
        "nn_structure": "grid over x, y (mpt_rrt_last_nn)",
        "examined_per_query": round(examined, 2),
        "floor_per_query": round(fl, 2),
        "floor_median": float(floor.median().item()),
        "examined_over_floor": round(examined / fl, 3) if fl > 0 else None,
        "nn_query_ms": round(times["nn_query"], 4),
        "nn_build_ms": round(times["nn_build"], 4),
        "spot_check_nearest": spot_ok,
        "definition": "floor = tree nodes whose (dx^2 + dy^2) is below the query's final best squared distance: "
                      "any index pruning on x, y alone must examine them",
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
