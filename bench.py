"""Benchmark: valid RRT edge extensions/s (collision + NN), BASELINE.json config 2.

Workload (one "step" = one batched RRT round on the device, motionplanningtoolkit_amd.RRTEngine):
  blimp agent (blimp.3ds, all 1355 triangles) in the single-room environment (model.dae,
  316 triangles), tree of 100k synthetic states ~ U(Blimp::getStateVarRanges), K = 65536
  extensions per round: uniform sample -> exact 1-NN over the 100k-node tree -> randomSteer
  -> getPoses -> FCL-semantics collision -> ordered append of the collision-free edges.
  The tree is reset to its 100k base at the start of every round (inside the timed step)
  so every round does identical work.

Multi-GPU: one process per GPU (torchrun), each rank runs its own seed (independent
trees, weak scaling); the only collective is the final max/sum reduction of timings and
counters (RCCL), outside the data path.

Prints ONE JSON line (rank 0).  See DESIGN.md "Measurement" for the roofline definition.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 (vector = matrix), AMD public spec; FMA counted as 2
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=65536, help="extensions per round (K)")
    ap.add_argument("--tree", type=int, default=100_000, help="tree nodes at the start of each round (N0)")
    ap.add_argument("--seed", type=int, default=1000)
    ap.add_argument("--workload", default="blimp", choices=["blimp", "snake"],
                    help="blimp = BASELINE config 2 (default); snake = config 3 (snake_trailers, 11 links, corridor)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample length")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--stage-every", type=int, default=8,
                    help="record the per-stage hipEvents on every n-th timed round (0: none); each recorded "
                         "round pays ~34 us of event packets, so they sample the timed region")
    ap.add_argument("--nn", default="auto", choices=["grid", "brute", "auto", "tree"], help="engine NN structure")
    ap.add_argument("--ppc", type=float, default=0.0,
                    help="grid points per cell (0: the engine's default, 2 floored by the expected NN distance)")
    ap.add_argument("--traffic", default=None, help="pmc_summary.json (default: latest profiles/r*/)")
    ap.add_argument("--seeds", type=int, default=0,
                    help="config 5: this many independent blimp RRTs (seed_base + i) sharded over the ranks "
                         "(0 = config 2, one 100k-node tree per rank)")
    ap.add_argument("--seed-batch", type=int, default=4096, help="config 5: extensions per seed per round")
    ap.add_argument("--streams", type=int, default=32, help="config 5: HIP streams the seeds' rounds rotate over")
    ap.add_argument("--no-joint-nn", action="store_true",
                    help="config 5: each seed queries its own tree (default: one joint NN launch per round, "
                         "mpt_rrt_step_many)")
    ap.add_argument("--joint-groups", type=int, default=1,
                    help="config 5: split the seeds into this many step_many groups, each on its own streams "
                         "and joint stream, so one group's NN launch overlaps another's build / collide")
    ap.add_argument("--launch-threads", type=int, default=1,
                    help="config 5: host threads issuing the seeds' rounds (thread t drives streams t, t+T, ...)")
    return ap.parse_args()


def cpu_baseline(sc, tree, K_gpu, seed, target_s):
    """The oracle (C port of the reference's FCL+FLANN semantics) on the host: the same
    round on a bounded sample of extensions, 1 thread (the reference is single-threaded),
    kd-tree NN built once per round (FLANN KDTreeSingleIndex-like), AABB-tree collision."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc

    bvh = orc.BVH(sc.env_tris)
    n0 = tree.shape[0]

    def run(K, threads):
        nodes = np.zeros((n0 + K, sc.dim))
        nodes[:n0] = tree
        par = np.zeros(n0 + K, np.int32)
        t = time.perf_counter()
        n, _, _ = orc.engine_step(sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, seed, 0, K, bvh, sc.env_tf,
                                  sc.agent_tris, nodes, par, n0, nthreads=threads, use_kdtree=True)
        return time.perf_counter() - t, n - n0

    # per-round fixed cost (the kd-tree build) + per-extension cost, from two short runs
    t_a, _ = run(256, 1)
    t_b, _ = run(1024, 1)
    per = max((t_b - t_a) / 768, 1e-7)
    fixed = max(t_a - 256 * per, 0.0)
    K = int(min(max((target_s - fixed) / per, 256), K_gpu))
    t1, valid1 = run(K, 1)
    threads = os.cpu_count() or 1
    threads = min(threads, 16)
    tn, validn = run(K, threads)
    return {
        "value": valid1 / t1, "unit": "valid extensions/s", "cores": 1, "kind": "port",
        "sample": f"{K} extensions of the same {sc.name} round ({n0}-node tree, kd-tree NN built per round, "
                  f"AABB-tree + FCL tri-tri SAT), oracle/mpt_oracle.c, {t1:.2f} s",
        "all_cores": {"value": validn / tn, "cores": threads, "seconds": round(tn, 3)},
        "cpu": _cpu_model(),
    }


# Stage -> the kernel that does its work (kernel names as rocprofv3 reports them).
STAGE_KERNEL = {"nn_query": "k_grid_nn1_runs", "collide_pairs": "k_pairs", "collide_cands": "k_cands",
                "collide_narrow": "k_narrow", "nn_build": "k_grid_scatter", "steer": "k_steer",
                "sample": "k_sample", "append": "k_append"}


def stage_bytes(stage, c, K, n0, d, pmax, nn_mode="grid"):
    """Algorithmic bytes one launch of the stage must touch (DESIGN.md "Measurement"): the
    inputs it reads and outputs it writes, each counted once per use, from the counters
    of the round (c = RRTEngine.collide_stats)."""
    if stage == "nn_query":  # queries + results + examined points (coords, id) + cell ranges
        # grid: a cell's (start, count) pair; tree: a box's float lo / hi over d dims
        per_cell = 8 * d if nn_mode == "tree" else 8
        return K * (8 * d + 12) + c["nn_points"] * (8 * d + 4) + c["nn_cells"] * per_cell
    if stage == "collide_pairs":  # poses, cluster records, env tree items tested, pair words
        return c["units"] * 96 + c["cluster_threads"] * 64 + c["node_tests"] * 32 + c["pair_tests"] * 4
    if stage == "collide_cands":  # per header: header, pose, 64 agent triangles; pairs; candidates
        return c["cluster_transforms"] * (32 + 96 + 64 * 72) + c["pair_tests"] * (4 + 32) + c["candidates"] * 12
    if stage == "collide_narrow":  # per candidate: itself, pose, agent triangle, env triangle record
        return c["candidates"] * (12 + 96 + 72 + 384)
    if stage == "nn_build":  # read the tree, write it in cell order with ids, cell counts
        return n0 * (2 * 8 * d + 12)
    if stage == "steer":  # nn id, tree node, end state, poses
        return K * (4 + 16 * d + 96 * pmax + 4)
    if stage == "sample":
        return K * 8 * d
    if stage == "append":
        return K * (1 + 8 * d + 4) * 2
    return None


NN_KERNEL = {"grid": "k_grid_nn1_runs", "tree": "k_tree_nn1", "brute": "k_knn1"}


def roofline(per_launch, cst, K, n0, d, pmax, nn_mode, traffic_path):
    """Roofline of the round's dominant kernel: achieved = its algorithmic bytes per launch
    / its hipEvent-measured duration (per-stage events on the engine's stream); every
    stage's figure is listed under `stages`."""
    stages = {}
    kernels = dict(STAGE_KERNEL, nn_query=NN_KERNEL.get(nn_mode, STAGE_KERNEL["nn_query"]))
    if nn_mode == "grid":  # the instantiation (its PMC row): the XCD-slab variant for d >= 15
        kernels["nn_query"] = f"k_grid_nn1_runs_xcd<{d}," if d >= 15 else f"k_grid_nn1_runs<{d},"
    if nn_mode == "tree":
        kernels["nn_build"] = "k_pt_gather"
    for s in kernels:
        ms = per_launch.get(s, 0.0)
        b = stage_bytes(s, cst, K, n0, d, pmax, nn_mode)
        if ms <= 0 or b is None:
            continue
        gbs = b / (ms * 1e-3) / 1e9
        stages[s] = {"kernel": kernels[s], "ms": round(ms, 4), "bytes": int(b), "achieved_gbs": round(gbs, 1),
                     "frac": round(gbs / HBM_PEAK_GBS, 4)}
        t = pmc_traffic(traffic_path, kernels[s])
        if t is not None:  # measured HBM bytes per launch (rocprofv3 PMC) over the same time
            stages[s]["traffic"] = t
            stages[s]["traffic_gbs"] = round(t / (ms * 1e-3) / 1e9, 1)
    if not stages:  # no stage timing recorded (--stage-every 0)
        return {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                "traffic": None, "stages": {}, "work_per_round": cst}
    dominant = max(stages, key=lambda s: stages[s]["ms"])
    st = stages[dominant]
    traffic = pmc_traffic(traffic_path, st["kernel"])
    # achieved counts algorithmic bytes, which caches (LDS, L2, MALL) may serve;
    # traffic_gbs is the measured HBM rate of the same launches, the honest distance to the roof
    out = {"bound": "hbm", "achieved": st["achieved_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": st["frac"], "traffic": traffic,
           "traffic_gbs": st.get("traffic_gbs"), "kernel": st["kernel"], "stage": dominant,
           "ms_per_launch": st["ms"], "algorithmic_bytes": st["bytes"], "stages": stages, "work_per_round": cst}
    if dominant == "nn_query" and nn_mode == "brute":
        flops = float(K) * n0 * 3 * d  # 3*d*N FP64 ops per query (sub, mul, add)
        tf = flops / (st["ms"] * 1e-3) / 1e12
        out.update({"bound": "mfma", "achieved": round(tf, 3), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(tf / FP64_PEAK_TFLOPS, 4), "kernel": "k_knn1",
                    "note": "FP64 VALU (FLANN's L2 op order is not a dot product, so no MFMA)"})
    return out


def pmc_traffic(path, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (scripts/profile.sh + scripts/pmc_summary.py), or None."""
    if not path:
        import glob

        cands = sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "pmc_summary.json")))
        path = cands[-1] if cands else None
    try:
        summ = json.load(open(path))
    except (OSError, ValueError, TypeError):
        return None
    for name, v in summ.items():
        if kernel in name:
            return v["hbm_bytes_per_launch"]
    return None


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def run_seeds(args, world, rank, dist, torch, mpt, multiseed, scenes):
    """BASELINE config 5: `args.seeds` independent blimp RRTs, each its own engine and tree grown
    from the blimp start state, `args.seed_batch` extensions per seed per round; rank r runs
    the contiguous shard multiseed.shard_seeds(seeds, world, r).  Total work is fixed as the
    GPU count grows (strong scaling).  A seed's tree depends only on its seed (counter-based
    RNG), so the digest of all trees is the same at every GPU count."""
    sc = scenes.blimp_scenario("all")
    env = mpt.Environment(sc.env_tris, sc.env_tf)
    agent = mpt.AgentMesh(sc.agent_tris)
    mine = list(multiseed.shard_seeds(args.seeds, world, rank))
    K = args.seed_batch
    rounds = args.warmup + args.steps
    # collision-free start at rest in the middle of the room (model.dae spans (0,0,0)-(177,138,114);
    # blimp.inst's start (0,0,0) is the room's corner, inside its walls)
    start = np.array([[88.6, 68.9, 57.1, 0.0, 0.0, 0.0, 0.0]])
    engines = []
    for i in mine:
        e = mpt.RRTEngine(env, agent, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, 1 + (rounds + 2) * K,
                          args.seed + i)
        e.add_nodes(start)
        e.set_nn(args.nn, args.ppc)
        engines.append(e)
    streams = [torch.cuda.Stream() for _ in range(max(1, min(args.streams, len(engines))))]
    if engines:
        engines[0].enable_timing(True)

    # a seed round is ~25 small launches, so 256 seeds from one host thread are launch-bound;
    # T threads each drive the engines of streams t, t + T, ... (ctypes drops the GIL)
    T = max(1, min(args.launch_threads, len(streams)))
    groups = [[(e, streams[j % len(streams)]) for j, e in enumerate(engines) if (j % len(streams)) % T == t]
              for t in range(T)]

    def drive(g):
        for e, s in g:
            e.step(K, s)

    pool = None
    if T > 1:
        from concurrent.futures import ThreadPoolExecutor

        dev = torch.cuda.current_device()
        pool = ThreadPoolExecutor(T, initializer=torch.cuda.set_device, initargs=(dev,))

    joint = torch.cuda.Stream()
    eng_streams = [streams[j % len(streams)] for j in range(len(engines))]
    # groups: contiguous slices of engines, group g on streams [g*S/G, (g+1)*S/G) + its own joint stream
    G = max(1, min(args.joint_groups, len(streams), len(engines)))
    gsz = -(-len(engines) // G)
    spg = max(1, len(streams) // G)
    jgroups = []
    for g in range(G):
        eg = engines[g * gsz:(g + 1) * gsz]
        sg = streams[g * spg:(g + 1) * spg]
        if eg:
            jgroups.append((eg, [sg[j % len(sg)] for j in range(len(eg))], joint if g == 0 else torch.cuda.Stream()))

    def round_():
        if not args.no_joint_nn:
            for eg, ss, js in jgroups:
                mpt.step_many(eg, K, ss, js)
        elif pool is None:
            drive(groups[0])
        else:
            for f in [pool.submit(drive, g) for g in groups]:
                f.result()

    for _ in range(args.warmup):
        round_()
    torch.cuda.synchronize()
    c0 = [e.counters() for e in engines]
    ktimes = {}
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        round_()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    c1 = [e.counters() for e in engines]
    valid = sum(b["valid"] - a["valid"] for a, b in zip(c0, c1))
    checked = sum(b["checked"] - a["checked"] for a, b in zip(c0, c1))
    elapsed, (valid, checked) = multiseed.reduce_run(dist, elapsed, [valid, checked], "cuda")
    digests = {}
    for i, e, c in zip(mine, engines, c1):
        st, par = e.read_tree(c["nodes"])
        digests[i] = multiseed.tree_digest(st, par)
    digests = multiseed.gather_digests(dist, digests)
    if rank != 0:
        return None
    # seed 0's engine: one more round with stage timing and work counters, outside the timed region
    e0 = engines[0]
    n_before = e0.counters()["nodes"]
    if args.no_joint_nn:
        e0.collide_stats(True)
        e0.step(K, streams[0])
        torch.cuda.synchronize()
        cst = e0.collide_stats(False)
        per_launch = e0.kernel_times()
        roof = roofline(per_launch, cst, K, n_before, sc.dim, e0.info()["pmax"], e0.last_nn(), args.traffic)
    else:
        # all seeds: one round with work counters on (summed for the joint launch's bytes), then
        # one with them off and the joint NN launch timed by hipEvents on its stream
        for e in engines:
            e.collide_stats(True)
        mpt.step_many(engines, K, eng_streams, joint)
        torch.cuda.synchronize()
        csts = [e.collide_stats(False) for e in engines]
        mpt.step_many(engines, K, eng_streams, joint)
        torch.cuda.synchronize()
        jms = mpt.joint_nn_ms()
        cst = csts[0]
        per_launch = dict(e0.kernel_times())
        nn_bytes = sum(stage_bytes("nn_query", c, K, n_before, sc.dim, e0.info()["pmax"], "tree") for c in csts)
        per_launch.pop("nn_query", None)
        roof = roofline(per_launch, cst, K, n_before, sc.dim, e0.info()["pmax"], e0.last_nn(), args.traffic)
        gbs = nn_bytes / (jms * 1e-3) / 1e9
        nn = {"kernel": "k_tree_nn1_jobs<7,", "ms": round(jms, 4), "bytes": int(nn_bytes),
              "achieved_gbs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
              "launch": f"one launch for all {len(engines)} seeds' {K} queries"}
        t = pmc_traffic(args.traffic, nn["kernel"])
        if t is not None:
            nn["traffic"], nn["traffic_gbs"] = t, round(t / (jms * 1e-3) / 1e9, 1)
        roof["stages"]["nn_query"] = nn
        roof.update({"achieved": nn["achieved_gbs"], "frac": nn["frac"], "traffic": nn.get("traffic"),
                     "traffic_gbs": nn.get("traffic_gbs"), "kernel": nn["kernel"], "stage": "nn_query",
                     "ms_per_launch": nn["ms"], "algorithmic_bytes": nn["bytes"],
                     "work_nn_all_seeds": {"nn_points": sum(c["nn_points"] for c in csts),
                                           "nn_boxes": sum(c["nn_cells"] for c in csts)}})
    import hashlib

    all_digest = hashlib.sha256("".join(digests[i] for i in sorted(digests)).encode()).hexdigest()
    return {
        "metric": "valid RRT edge extensions/sec (collision+NN) per node, 1/2/4/8 MI355X",
        "value": valid / elapsed,
        "unit": "valid extensions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (uniform samples over Blimp::getStateVarRanges; meshes from the reference)",
        "config": {"workload": f"config 5: {args.seeds} independent blimp RRTs (1355-tri blimp vs model.dae) "
                               f"grown from the start state, {K} extensions per seed per round",
                   "seeds": args.seeds, "seed_base": args.seed, "extensions_per_seed_round": K,
                   "rounds_before_timing": args.warmup, "streams_per_gpu": len(streams), "launch_threads": T,
                   "joint_nn": not args.no_joint_nn, "joint_groups": G,
                   "parallelism": f"seeds sharded over {world} GPU(s)"},
        "checked_per_s": checked / elapsed,
        "valid_fraction": valid / max(checked, 1),
        "seeds_digest": all_digest,
        "roofline": roof,
        "cpu_baseline": None,
    }


def main():
    args = parse()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import motionplanningtoolkit_amd as mpt
    from motionplanningtoolkit_amd import multiseed, scenes

    mpt.init(local)
    torch.cuda.set_device(local)
    stream = torch.cuda.current_stream()
    if args.seeds > 0:
        out = run_seeds(args, world, rank, dist, torch, mpt, multiseed, scenes)
        if out is not None:
            print(json.dumps(out))
        if dist:
            dist.destroy_process_group()
        return

    if args.workload == "snake":
        sc = scenes.snake_scenario("corridor")
        workload = (f"snake.inst: snake_trailers ({sc.links} unit-box links, T=10) in the synthetic corridor "
                    f"({sc.env_tris.shape[0]} tris), batched RRT round over a {args.tree}-node tree")
    else:
        sc = scenes.blimp_scenario("all")
        workload = ("blimp.inst: blimp (1355 tris) vs single-room env (model.dae, 316 tris), "
                    f"batched RRT round over a {args.tree}-node tree")
    seed = multiseed.rank_seed(args.seed, rank)
    rng = np.random.default_rng(seed)
    n0, K = args.tree, args.batch
    tree = rng.uniform(sc.ranges[:, 0], sc.ranges[:, 1], size=(n0, sc.dim))
    env = mpt.Environment(sc.env_tris, sc.env_tf)
    agent = mpt.AgentMesh(sc.agent_tris)
    eng = mpt.RRTEngine(env, agent, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, n0 + K, seed)
    eng.add_nodes(tree)
    eng.set_nn(args.nn, args.ppc)
    eng.enable_timing(True)

    def round_():
        eng.set_size(n0, stream)
        eng.step(K, stream)

    for _ in range(args.warmup):
        round_()
    torch.cuda.synchronize()
    c0 = eng.counters()
    eng.kernel_times_sum()  # drop the warm-up rounds' stage times

    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if args.stage_every != 1:
            eng.enable_timing(args.stage_every > 0 and i % args.stage_every == 0)
        round_()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.enable_timing(True)
    c1 = eng.counters()
    valid = c1["valid"] - c0["valid"]
    checked = c1["checked"] - c0["checked"]

    elapsed, (valid, checked) = multiseed.reduce_run(dist, elapsed, [valid, checked], "cuda")

    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return

    steps = args.steps
    # hipEvents on the launch stream, recorded every timed round into the engine's event ring
    # and read only now (no host sync inside the timed region)
    ktimes, kt_rounds = eng.kernel_times_sum()
    per_launch = {k: v / max(kt_rounds, 1) for k, v in ktimes.items()}
    # one more round, outside the timed region, with the collision work counters on
    eng.collide_stats(True)
    round_()
    cst = eng.collide_stats(False)
    roof = roofline(per_launch, cst, K, n0, sc.dim, eng.info()["pmax"], eng.last_nn(), args.traffic)

    out = {
        "metric": "valid RRT edge extensions/sec (collision+NN) per node, 1/2/4/8 MI355X",
        "value": valid / elapsed,
        "unit": "valid extensions/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * elapsed / steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": f"synthetic (uniform samples and tree states over the {args.workload}'s getStateVarRanges; "
                "meshes from the reference)",
        "config": {"workload": workload,
                   "tree_nodes": n0, "extensions_per_round": K, "seed_base": args.seed, "nn_index": args.nn,
                   "parallelism": f"independent seeds x{world}"},
        "checked_per_s": checked / elapsed,
        "valid_fraction": valid / max(checked, 1),
        "kernel_ms_per_round": {k: round(v, 4) for k, v in per_launch.items()},
        "stage_timing": f"hipEvents on {kt_rounds} of the {steps} timed rounds (every {args.stage_every})",
        "roofline": roof,
    }
    if not args.no_cpu and world == 1:
        out["cpu_baseline"] = cpu_baseline(sc, tree, K, seed, args.cpu_seconds)
    else:
        out["cpu_baseline"] = None
    print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
