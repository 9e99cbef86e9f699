"""Benchmark: valid RRT edge extensions/s (collision + NN), BASELINE.json config 2.

Workload (one "step" = one batched RRT round on the device, motionplanningtoolkit_amd.RRTEngine):
  blimp agent (blimp.3ds, all 1355 triangles) in the single-room environment (model.dae,
  316 triangles), tree of 100k synthetic states ~ U(Blimp::getStateVarRanges), K = 65536
  extensions per round: uniform sample -> exact 1-NN over the 100k-node tree -> randomSteer
  -> getPoses -> FCL-semantics collision -> ordered append of the collision-free edges.
  The tree is reset to its 100k base at the start of every round (inside the timed step)
  so every round does identical work.
  --workload blimp-room: the same with the sampling box = the room's box, so every pose is
  inside the room and reaches the narrow phase (the collision-heavy variant of config 2);
  --workload snake: config 3; --seeds N: config 5 (N independent RRTs).

Multi-GPU: one process per GPU (torchrun), each rank runs its own seed (independent
trees, weak scaling); the only collective is the final max/sum reduction of timings and
counters (RCCL), outside the data path.

Prints ONE JSON line (rank 0).  Roofline: per stage, compulsory bytes (every
input and output of the launch once) / hipEvent time against the HBM peak, the measured HBM
traffic of the same kernel (rocprofv3 FETCH_SIZE / WRITE_SIZE, profiles/<latest>/) against
the same peak, their ratio, and the FP64 (collision kernels) or LDS (k_pairs) fraction.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector peak (AMD public spec; FMA counted as 2)
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md §HBM: 8.0 TB/s spec
LDS_PEAK_GBS = 150_000.0  # MI355X_MICROARCH.md §LDS: ~150 TB/s aggregate ds_read_b64/b128, every CU


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU).  Without torchrun's WORLD_SIZE, N > 1 starts torch.distributed.run "
                         "with N ranks as a child process (before any GPU call) and exits with its code; under "
                         "torchrun it must equal WORLD_SIZE (default: WORLD_SIZE, else 1)")
    ap.add_argument("--detail", default=os.path.join(REPO, "gpurun_out", "bench_detail.json"),
                    help="where rank 0 writes the full line (every stage table, every leg); the printed line is "
                         "the condensed one (empty: none)")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=65536, help="extensions per round (K)")
    ap.add_argument("--tree", type=int, default=100_000, help="tree nodes at the start of each round (N0)")
    ap.add_argument("--seed", type=int, default=1000)
    ap.add_argument("--workload", default="blimp", choices=["blimp", "blimp-room", "snake"],
                    help="blimp = BASELINE config 2 (default); blimp-room = config 2 with every pose inside the room "
                         "(collision-heavy); snake = config 3 (snake_trailers, 11 links, corridor)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample length")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-variants", action="store_true",
                    help="skip the secondary workloads' legs (config 2 at N=1 runs them by default, each in a "
                         "process of its own, and reports them under `variants`)")
    ap.add_argument("--stage-every", type=int, default=16,
                    help="record the per-stage hipEvents on every n-th timed round (0: none); a recorded round "
                         "pays ~60-80 us of event packets (config 2: 170 us a round with none, "
                         "scripts/host_rate.py, 178 us with every 8th), so they sample the timed region")
    ap.add_argument("--nn", default="auto", choices=["grid", "brute", "auto", "tree"], help="engine NN structure")
    ap.add_argument("--ppc", type=float, default=0.0,
                    help="grid points per cell (0: the engine's default, 2 floored by the expected NN distance)")
    ap.add_argument("--traffic", default=None, help="pmc_summary.json (default: latest profiles/r*/)")
    ap.add_argument("--seeds", type=int, default=0,
                    help="config 5: this many independent blimp RRTs (seed_base + i) sharded over the ranks "
                         "(0 = config 2, one 100k-node tree per rank)")
    ap.add_argument("--seed-batch", type=int, default=4096, help="config 5: extensions per seed per round")
    ap.add_argument("--seed-start", default="walls", choices=["walls", "centre"],
                    help="config 5: start each seed near a wall of the room (default, so trees reach the walls "
                         "and collide) or at the room's centre")
    ap.add_argument("--streams", type=int, default=0,
                    help="config 5: HIP streams the seeds' per-engine rounds rotate over (0, the default: every engine "
                         "on its group's joint stream -- a joint round then joins no other stream; 32 streams cost "
                         "~0.45 ms a round of event joins at 32 seeds)")
    ap.add_argument("--no-joint-nn", action="store_true",
                    help="config 5: each seed builds and queries its own tree (default: one joint build and one "
                         "joint NN launch per round, mpt_rrt_step_many)")
    ap.add_argument("--joint-groups", type=int, default=1,
                    help="config 5: split the seeds into this many step_many groups, each on its own streams "
                         "and joint stream, so one group's NN launch overlaps another's build / collide")
    ap.add_argument("--launch-threads", type=int, default=1,
                    help="config 5 with --no-joint-nn: host threads issuing the seeds' rounds")
    ap.add_argument("--c5-seeds", type=int, default=256,
                    help="the config-5 leg (every run without --seeds): seeds over all ranks (BASELINE config 5: "
                         "256, contiguous shards, 32 per GPU at 8 GPUs)")
    ap.add_argument("--c5-steps", type=int, default=C5_STEPS, help="the config-5 leg's timed rounds")
    ap.add_argument("--c5-warmup", type=int, default=C5_WARMUP, help="the config-5 leg's untimed rounds before them")
    return ap.parse_args()


# config 5 is measured at these rounds in every leg (the 32- and 256-seed legs of an N = 1 run,
# the in-world leg of an N > 1 run, and the PMC profiles their traffic columns come from), so
# their trees have the same sizes and their per-GPU ratio compares like with like
C5_STEPS, C5_WARMUP = 25, 5


# ----------------------------------------------------------------------------- CPU baseline

def cpu_cores():
    """CPUs this job may use: the affinity set, capped by the cgroup CPU quota (the GPU box's
    job gets a 16-CPU quota of a 256-CPU host; nproc there reports 16 via OMP_NUM_THREADS)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(int(q) // int(p)))
    except (OSError, ValueError):
        pass
    return (min(aff, quota) if quota else aff), {"affinity_cpus": aff, "cgroup_quota_cpus": quota,
                                                 "host_cpus": os.cpu_count()}


def _oracle_native():
    """The oracle compiled for this host (-O3 -march=native) into a scratch directory; the
    portable -O3 build if the compiler is missing."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc

    out = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"mpt_oracle_native_{os.getpid()}")
    try:
        path = orc.build_native(out)
        orc.lib(path)
        flags = "-O3 -march=native -ffp-contract=off -fopenmp"
    except (OSError, subprocess.CalledProcessError):
        orc.lib()
        flags = "-O3 -ffp-contract=off -fopenmp (portable build; native build failed)"
    return orc, flags


def cpu_baseline(sc, tree, K_gpu, seed, target_s):
    """The oracle (C restatement of the reference's FCL + FLANN semantics) on the host, timed
    in the same run, three legs:
      * all cores: the GPU's round on a bounded sample of its extensions (kd-tree NN built once
        per round, AABB-tree + FCL tri-tri SAT collision), OpenMP over the extensions -- `value`;
      * 1 core: the same sample single-threaded (the reference is single-threaded);
      * FLANN 1.8.4 rebuild per insert: the reference's own loop, one extension at a time from
        the same 100k-node tree, the kd-tree rebuilt after every insertion
        (flannkdtreewrapper.hpp:35 addPoints -> buildIndex), 1 core."""
    orc, flags = _oracle_native()
    cores, core_info = cpu_cores()
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
    K = int(min(max((0.45 * target_s - fixed) / per, 256), K_gpu))
    t1, valid1 = run(K, 1)
    tn, validn = run(K, cores)
    # the reference's sequential loop with FLANN 1.8.4's rebuild per insert, ~0.4 of the budget
    nodes = np.zeros((n0 + 100_000, sc.dim))
    nodes[:n0] = tree
    par = np.zeros(nodes.shape[0], np.int32)
    v_seq, tried, s_seq = orc.rrt_seq_rebuild(sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, seed, 0, bvh,
                                              sc.env_tf, sc.agent_tris, nodes, par, n0, 100_000, 0.4 * target_s)
    return {
        "value": validn / tn, "unit": "valid extensions/s", "cores": cores, "kind": "port",
        "sample": f"{K} extensions of the same {sc.name} round ({n0}-node tree, kd-tree NN built per round, "
                  f"AABB-tree + FCL tri-tri SAT), oracle/mpt_oracle.c, OpenMP over {cores} cores, {tn:.2f} s",
        "compile_flags": flags,
        "cpu": _cpu_model(), **core_info,
        "single_core": {"value": valid1 / t1, "cores": 1, "seconds": round(t1, 3)},
        "flann_rebuild_per_insert": {
            "value": v_seq / s_seq if s_seq > 0 else None, "cores": 1, "extensions": tried, "valid": v_seq,
            "seconds": round(s_seq, 3),
            "note": f"the reference's one-at-a-time loop from the same {n0}-node tree with a full kd-tree "
                    "rebuild after every insertion (FLANN 1.8.4 addPoints, flannkdtreewrapper.hpp:35)"},
    }


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# ----------------------------------------------------------------------------- roofline

# Stage -> the kernel that does its work (names as rocprofv3 reports them).
STAGE_KERNEL = {"nn_query": "k_grid_nn1_runs", "collide_pairs": "k_pairs", "collide_cands": "k_cands",
                "collide_narrow": "k_narrow", "nn_build": "k_grid_scatter", "steer": "k_steer",
                "sample": "k_sample", "append": "k_append"}
NN_KERNEL = {"grid": "k_grid_nn1_runs", "tree": "k_ct_nn1", "brute": "k_knn1"}


def geometry(sc, env):
    """Sizes the compulsory-byte model needs: env / agent triangles, agent clusters (<= 64
    triangles each, mpt_agent_create), env tree items (one per triangle + buckets of <= 16)."""
    te = int(env.info()["triangles"])
    ta = int(sc.agent_tris.shape[0])
    return {"env_tris": te, "agent_tris": ta, "clusters": max(1, -(-ta // 64)), "env_items": te + -(-te // 8),
            "links": int(getattr(sc, "links", 1) or 1)}


def inc_build_bytes(n, m, d):
    """The cell tree's round (cell_tree.hip) over trees holding n points in total after it, m
    of them new: the new rows read and their (code, row) pairs written and read back by the
    sort; the touched buckets (at most m, 8 slots of row, id and 16-byte code each) read and
    rewritten; the directory (about n / 4 entries: buckets hold 1..8 points) read and written
    by the merge; the box levels above it (about n_dir * 8 / 7 nodes of 2d floats, a meta word
    and a 16-byte code) written once and read once by the level above."""
    slot = 8 * d + 4 + 16
    n_dir = n // 4
    nodes = n_dir * 8 // 7
    return m * 8 * d + m * 24 * 2 + m * 8 * slot * 2 + n_dir * 20 * 2 + nodes * (8 * d + 4 + 16) * 2


def compulsory_bytes(stage, c, K, n0, d, pmax, geo, nn_mode):
    """Every input and output of one launch of the stage counted once (the HBM minimum);
    c = RRTEngine.collide_stats of one round."""
    rec = 8 * (d + 1) if d < 8 else 8 * d + 4  # grid point record (+ id)
    live = c["cluster_threads"] / geo["clusters"]  # (pose, link) units past k_steer's object cull
    if stage == "sample":
        return K * 8 * d
    if stage == "nn_build":
        if nn_mode == "tree":  # the incremental build (one round's K new points)
            return inc_build_bytes(n0, min(K, n0), d)
        return n0 * (8 * d + rec + 8) + (n0 // 2) * 12  # nodes in, records out, cell ids, counts / starts
    if stage == "nn_query":
        if nn_mode != "grid":
            # a pruned search over a tree that covers part of the sampling box (config 5: most
            # samples lie far from the tree and touch its boundary leaves only) need not read the
            # whole index: its queries and results (index bytes reported beside, index_bytes)
            return K * (8 * d + 12)
        return K * (8 * d + 12) + n0 * rec + (n0 // 2) * 4
    if stage == "steer":
        # ids, neighbour rows, end states, counts, verdict init; every (pose, link) unit's pose
        # and its FCL relative transform (96 B each, k_steer writes both); the live list
        units = K * pmax * geo.get("links", 1)
        return K * (4 + 8 * d + 8 * d + 4 + 1) + units * 96 * 2 + live * 4
    if stage == "collide_pairs":  # live poses, clusters, env tree, pair words, headers
        return live * 96 + geo["clusters"] * 64 + geo["env_items"] * 32 + c["pair_tests"] * 4 + c["cluster_transforms"] * 32
    if stage == "collide_cands":  # headers, pair words, poses, agent triangles, env boxes, candidates
        return (c["cluster_transforms"] * 32 + c["pair_tests"] * 4 + live * 96 + geo["agent_tris"] * 72
                + geo["env_items"] * 32 + c["candidates"] * 12)
    if stage == "collide_narrow":  # candidates, poses, agent triangles, env records, verdicts
        return c["candidates"] * 12 + live * 96 + geo["agent_tris"] * 72 + geo["env_tris"] * 384 + K
    if stage == "append":
        return K * (1 + 8 * d + 4) * 2
    return None


def fp64_flops(stage, c, geo):
    """FP64 work of the collision stages by SURVEY §8(d): 54 flops per agent triangle mapped
    (Q' = R Q + T), 750 per exact triangle-pair test, + the relative transform and box of a
    (unit, cluster) thread (~81)."""
    if stage == "collide_narrow":
        return 54.0 * c["candidates"] + 750.0 * c["tri_tests"]
    if stage == "collide_cands":
        return 54.0 * c["cluster_transforms"] * geo["agent_tris"] / geo["clusters"]
    if stage == "collide_pairs":
        return 81.0 * c["cluster_threads"]
    return None


def lds_bytes(stage, c, geo):
    """k_pairs reads every env tree item it tests from LDS (32 B) after each workgroup stages
    the tree (env_items * 32 B per 256-thread workgroup)."""
    if stage != "collide_pairs":
        return None
    return c["node_tests"] * 32.0 + (c["cluster_threads"] / 256.0) * geo["env_items"] * 32.0


def touched_bytes(stage, c, K, n0, d, pmax):
    """Bytes the stage touches through any level of the hierarchy (round 1's figure, kept
    for reference: examined points, tested tree items, candidate records)."""
    if stage == "nn_query":
        return K * (8 * d + 12) + c["nn_points"] * (8 * d + 4) + c["nn_cells"] * 8
    if stage == "collide_pairs":
        return c["units"] * 96 + c["cluster_threads"] * 64 + c["node_tests"] * 32 + c["pair_tests"] * 4
    if stage == "collide_cands":
        return c["cluster_transforms"] * (32 + 96 + 64 * 72) + c["pair_tests"] * (4 + 32) + c["candidates"] * 12
    if stage == "collide_narrow":
        return c["candidates"] * (12 + 96 + 72 + 384)
    return None


# workload -> the subdirectory of profiles/r*/ that holds its own PMC summary (the same kernel
# names move different bytes in each workload)
PMC_SUBDIR = {"blimp": "", "blimp-room": "room", "snake": "snake"}


def pmc_summary(path, workload="blimp"):
    if not path:
        import glob

        # config 5: the summary profiled at the same seed count (profiles/r*/c5_<seeds>/)
        sub = f"c5_{workload[5:]}" if workload.startswith("seeds") else PMC_SUBDIR.get(workload, "")
        cands = sorted(glob.glob(os.path.join(REPO, "profiles", "r[0-9][0-9]", sub, "pmc_summary.json")))
        path = cands[-1] if cands else None
    try:
        return json.load(open(path)), os.path.relpath(path, REPO)
    except (OSError, ValueError, TypeError):
        return {}, None


def pmc_traffic(summ, kernel):
    """Measured HBM bytes per launch of `kernel`: (2 * FETCH_SIZE + WRITE_SIZE) * 1024 from the
    committed rocprofv3 PMC summary (scripts/profile.sh + scripts/pmc_summary.py)."""
    for name, v in summ.items():
        if kernel in name:
            return v["hbm_bytes_per_launch"]
    return None


def pmc_traffic_sum(summ, subs):
    """Measured HBM bytes of a stage's launch chain: every summary entry whose kernel name
    contains one of `subs` (each entry once; template instances of one kernel all count),
    None when none is in the summary."""
    hits = [v["hbm_bytes_per_launch"] for name, v in summ.items() if any(s in name for s in subs)]
    return sum(hits) if hits else None


def stage_table(per_launch, cst, K, n0, d, pmax, geo, nn_mode, kernels, summ):
    stages = {}
    for s, kern in kernels.items():
        ms = per_launch.get(s, 0.0)
        b = compulsory_bytes(s, cst, K, n0, d, pmax, geo, nn_mode)
        if ms <= 0 or b is None:
            continue
        t = ms * 1e-3
        st = {"kernel": kern, "ms": round(ms, 4), "compulsory_bytes": int(b),
              "compulsory_gbs": round(b / t / 1e9, 1), "frac_hbm_compulsory": round(b / t / 1e9 / HBM_PEAK_GBS, 4)}
        tr = pmc_traffic(summ, kern)
        if tr is not None:
            st.update({"traffic": int(tr), "traffic_gbs": round(tr / t / 1e9, 1),
                       "frac_hbm_measured": round(tr / t / 1e9 / HBM_PEAK_GBS, 4),
                       "traffic_over_compulsory": round(tr / b, 2)})
        f = fp64_flops(s, cst, geo)
        if f is not None:
            st.update({"fp64_tflops": round(f / t / 1e12, 3), "frac_fp64": round(f / t / 1e12 / FP64_PEAK_TFLOPS, 4)})
        lb = lds_bytes(s, cst, geo)
        if lb is not None:
            st.update({"lds_gbs": round(lb / t / 1e9, 1), "frac_lds": round(lb / t / 1e9 / LDS_PEAK_GBS, 4)})
        tb = touched_bytes(s, cst, K, n0, d, pmax)
        if tb is not None:
            st["touched_bytes"] = int(tb)
        stages[s] = st
    return stages


# config 5's joint round: stage -> the kernels of its launch chain (rocprofv3 names), whose
# measured traffic per launch is summed (the collide chain runs once per collide sub-batch)
JOINT_STAGE_KERNELS = {
    "sample": ["k_sample_jobs"],
    "nn_build": ["k_ct_reset", "k_ct_ncodes", "k_ct_csort", "k_ct_crank", "k_ct_locate", "k_ct_segments",
                 "k_ct_apply", "k_ct_split_", "k_ct_dmerge", "k_ct_lflags", "k_ct_lgroup", "k_ct_levels"],
    "nn_query": ["k_ct_nn1_jobs"],
    "steer": ["k_steer_jobs"],
    "collide": ["k_pairs<", "k_scan_excl<mpt::ExpandHeaders", "k_cands", "k_narrow", "k_overflow"],
    "append": ["k_append_jobs"],
}


def joint_stage_table(times, c, K, nj, n_tot, d, pmax, geo, summ):
    """Per-stage roofline of one joint round of nj seeds (one launch per stage for all of
    them): compulsory bytes of all seeds' work, the measured traffic of every kernel of the
    stage's chain, FP64 of the collide stages; c = the seeds' summed work counters."""
    units = K * pmax * geo.get("links", 1)
    per_sub = max(1, (2 ** 25 // geo["clusters"]) // units)  # broad.hip kSplitChunkThreads
    n_sub = -(-nj // per_sub)
    stages = {}
    for s, ms in times.items():
        if ms <= 0:
            continue
        if s == "collide":
            b = sum(compulsory_bytes(x, c, K * nj, n_tot, d, pmax, geo, "tree")
                    for x in ("collide_pairs", "collide_cands", "collide_narrow"))
            f = sum(fp64_flops(x, c, geo) for x in ("collide_pairs", "collide_cands", "collide_narrow"))
        else:
            b = compulsory_bytes(s, c, K * nj, n_tot, d, pmax, geo, "tree")
            f = None
        if s == "nn_build":
            b = inc_build_bytes(n_tot + K * nj, K * nj, d)
        index_b = n_tot * (8 * d + 4) + (n_tot // 7) * 8 * d if s == "nn_query" else None
        if b is None:
            continue
        t = ms * 1e-3
        st = {"kernel": " + ".join(JOINT_STAGE_KERNELS.get(s, [])), "ms": round(ms, 4), "compulsory_bytes": int(b),
              "compulsory_gbs": round(b / t / 1e9, 1), "frac_hbm_compulsory": round(b / t / 1e9 / HBM_PEAK_GBS, 4),
              "launch": f"one joint launch per kernel for {nj} seeds x {K} extensions"
                        + (f" ({n_sub} collide sub-batches)" if s == "collide" else "")}
        if index_b:
            st["index_bytes"] = int(index_b)
        if s == "nn_query" and c.get("nn_points"):
            # work counters of the stats round (the same trees and queries): points examined and
            # boxes tested per query
            st["nn_points_per_query"] = round(c["nn_points"] / (K * nj), 2)
            st["nn_boxes_per_query"] = round(c["nn_cells"] / (K * nj), 2)
            st["nn_steps_per_query"] = round(c.get("nn_steps", 0) / (K * nj), 2)
        subs = JOINT_STAGE_KERNELS.get(s, [])
        tr = pmc_traffic_sum(summ, subs) if subs else None
        if tr is not None:
            tr *= n_sub if s == "collide" else 1
            st.update({"traffic": int(tr), "traffic_gbs": round(tr / t / 1e9, 1),
                       "frac_hbm_measured": round(tr / t / 1e9 / HBM_PEAK_GBS, 4),
                       "traffic_over_compulsory": round(tr / b, 2)})
        if f:
            st.update({"fp64_tflops": round(f / t / 1e12, 3), "frac_fp64": round(f / t / 1e12 / FP64_PEAK_TFLOPS, 4)})
        stages[s] = st
    return stages


def round_roof(stages, ms):
    """The whole round against the HBM roof: every stage's compulsory bytes (and, where every
    stage has a PMC row, its measured traffic) over the round's wall time per step."""
    if not stages or ms <= 0:
        return None
    t = ms * 1e-3
    b = sum(st["compulsory_bytes"] for st in stages.values())
    out = {"ms": round(ms, 4), "compulsory_bytes": int(b), "frac_hbm_compulsory": round(b / t / 1e9 / HBM_PEAK_GBS, 4)}
    tr = [st.get("traffic") for st in stages.values()]
    if all(x is not None for x in tr):
        out.update({"traffic": int(sum(tr)), "frac_hbm_measured": round(sum(tr) / t / 1e9 / HBM_PEAK_GBS, 4)})
    return out


def pmc_steady_us(summ, kernel):
    """The dominant kernel's steady-state duration in the committed profile (scripts/pmc_summary.py
    steady_us: the kernel trace of the same run as the counters, cold launches excluded)."""
    for name, v in summ.items():
        if kernel in name and v.get("steady_us"):
            return v["steady_us"], v.get("steady_launches")
    return None, None


def roofline_of(stages, dominant, work, summ_path, summ=None):
    """The contract's roofline object for the dominant stage: HBM-bound unless its FP64
    fraction is the larger one (then `fp64_valu` = the FP64 VALU roof; no MFMA: FCL's operation
    order is scalar FP64)."""
    if not stages or dominant not in stages:
        return {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None, "traffic": None,
                "stages": stages, "work_per_round": work}
    st = stages[dominant]
    out = {"bound": "hbm", "achieved": st["compulsory_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": st["frac_hbm_compulsory"], "traffic": st.get("traffic"), "traffic_gbs": st.get("traffic_gbs"),
           "frac_hbm_measured": st.get("frac_hbm_measured"), "traffic_over_compulsory": st.get("traffic_over_compulsory"),
           "kernel": st["kernel"], "stage": dominant, "ms_per_launch": st["ms"],
           "algorithmic_bytes": st["compulsory_bytes"], "pmc_source": summ_path}
    if st.get("frac_fp64", 0.0) > max(st["frac_hbm_compulsory"], st.get("frac_hbm_measured") or 0.0):
        out.update({"bound": "fp64_valu", "achieved": st["fp64_tflops"], "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": st["frac_fp64"], "note": "FP64 VALU roof (FCL's scalar operation order; no MFMA)"})
    us, nl = pmc_steady_us(summ or {}, st["kernel"])
    if us:
        # the same fraction from the profile's own steady-state duration: the line's hipEvent
        # time and the committed trace must agree
        out.update({"profile_us_per_launch": us, "profile_launches": nl,
                    "frac_from_profile": round(out["frac"] * st["ms"] * 1e3 / us, 4)})
    out["definition"] = ("achieved = compulsory bytes (each input and output of the launch once) / hipEvent time; "
                         "traffic = measured HBM bytes per launch (2*FETCH_SIZE + WRITE_SIZE, rocprofv3); "
                         "per-stage FP64 and LDS fractions under stages")
    out["stages"] = stages
    out["work_per_round"] = work
    return out


# ----------------------------------------------------------------------------- config 5

def seed_start(seed, env, agent, mpt, where):
    """Config 5 start state of a seed: at rest, collision-free, either at the room's centre or
    (default) 5.5-10 units from one of the room's four side walls (so the tree reaches walls
    within a few rounds and extensions collide); deterministic per seed."""
    if where == "centre":
        return np.array([[88.6, 68.9, 57.1, 0.0, 0.0, 0.0, 0.0]])
    rng = np.random.default_rng(seed)
    lo, hi = np.array([0.0, 0.0, 0.0]), np.array([177.16, 137.80, 114.17])
    for _ in range(64):
        p = rng.uniform(lo + 12, hi - 12)
        wall, dist = int(rng.integers(4)), rng.uniform(5.5, 10.0)
        if wall == 0:
            p[0] = lo[0] + dist
        elif wall == 1:
            p[0] = hi[0] - dist
        elif wall == 2:
            p[1] = lo[1] + dist
        else:
            p[1] = hi[1] - dist
        th = rng.uniform(0, 2 * np.pi)
        pose = np.r_[np.cos(th), np.sin(th), 0, -np.sin(th), np.cos(th), 0, 0, 0, 1, p].reshape(1, 1, 12)
        if mpt.collide_batch(env, [agent], pose, np.array([0, 1]))[0] == 0:
            return np.array([[p[0], p[1], p[2], th, 0.0, 0.0, 0.0]])
    return np.array([[88.6, 68.9, 57.1, 0.0, 0.0, 0.0, 0.0]])


def run_seeds(args, world, rank, dist, torch, mpt, multiseed, scenes):
    """BASELINE config 5: `args.seeds` independent blimp RRTs, each its own engine and tree grown
    from its start state, `args.seed_batch` extensions per seed per round; rank r runs the
    contiguous shard multiseed.shard_seeds(seeds, world, r).  Total work is fixed as the GPU
    count grows (strong scaling).  A seed's tree depends only on its seed (counter-based RNG),
    so the digest of all trees is the same at every GPU count."""
    sc = scenes.blimp_scenario("all")
    env = mpt.Environment(sc.env_tris, sc.env_tf)
    agent = mpt.AgentMesh(sc.agent_tris)
    mine = list(multiseed.shard_seeds(args.seeds, world, rank))
    K = args.seed_batch
    rounds = args.warmup + args.steps
    engines = []
    for i in mine:
        e = mpt.RRTEngine(env, agent, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, 1 + (rounds + 2) * K,
                          args.seed + i)
        e.add_nodes(seed_start(args.seed + i, env, agent, mpt, args.seed_start))
        e.set_nn(args.nn, args.ppc)
        engines.append(e)
    streams = [torch.cuda.Stream() for _ in range(max(1, min(max(args.streams, 1), len(engines))))]
    if engines:
        engines[0].enable_timing(True)

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

    # step_many groups: contiguous slices of engines, group g on streams [g*S/G, (g+1)*S/G) and
    # its own joint stream (the joint job tables belong to the joint stream)
    G = max(1, min(args.joint_groups, len(streams), len(engines)))
    gsz = -(-len(engines) // G)
    spg = max(1, len(streams) // G)
    jgroups = []
    for g in range(G):
        eg = engines[g * gsz:(g + 1) * gsz]
        sg = streams[g * spg:(g + 1) * spg]
        if eg:
            js = torch.cuda.Stream()
            # --streams 0: every engine on its group's joint stream (a joint round then joins no
            # other stream)
            jgroups.append((eg, [sg[j % len(sg)] if args.streams > 0 else js for j in range(len(eg))], js))

    def round_():
        if not args.no_joint_nn:
            for eg, ss, js in jgroups:
                mpt.step_many(eg, K, ss, js)
        elif pool is None:
            drive(groups[0])
        else:
            for f in [pool.submit(drive, g) for g in groups]:
                f.result()

    # The process's one-time HIP start-up before it: the joint round's kernels launched once (a
    # throwaway two-engine group on its own joint stream) and the streams' first work.  The first
    # launch of each kernel in a process and a stream's first work cost ~13 ms (scripts/
    # scratch_rounds.py: round 0 of 32 seeds 13.4 ms cold, 0.76 ms warm) -- once per process, not
    # per planner run -- so from_scratch measures the planner's rounds, and process_warmup_s
    # reports the start-up beside it.
    t_warm = time.perf_counter()
    for s_ in streams + [js for _, _, js in jgroups]:
        with torch.cuda.stream(s_):
            torch.zeros(1, device="cuda").add_(1)
    if not args.no_joint_nn and engines:
        tmp = []
        for i in range(2):
            e = mpt.RRTEngine(env, agent, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, 1 + 2 * K, args.seed + i)
            e.add_nodes(seed_start(args.seed + i, env, agent, mpt, args.seed_start))
            e.set_nn(args.nn, args.ppc)
            tmp.append(e)
        ws = torch.cuda.Stream()
        mpt.step_many(tmp, K, [ws] * 2, ws)
        torch.cuda.synchronize()
        for e in tmp:
            e.close()
        mpt.joint_release(ws)
    torch.cuda.synchronize()
    process_warmup = time.perf_counter() - t_warm
    # from scratch: every round from the seeds' start states (the first rounds' index
    # reservations included), then the timed rounds continue the same trees
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t_scratch = time.perf_counter()
    for _ in range(args.warmup):
        round_()
    torch.cuda.synchronize()
    c0 = [e.counters() for e in engines]
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host = 0.0
    for i in range(args.steps):
        if engines and args.stage_every != 1:
            # the joint round's stage events on every n-th timed round only (as config 2)
            engines[0].enable_timing(args.stage_every > 0 and i % args.stage_every == 0)
        h0 = time.perf_counter()
        round_()
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    scratch = t1 - t_scratch
    c1 = [e.counters() for e in engines]
    valid = sum(b["valid"] - a["valid"] for a, b in zip(c0, c1))
    checked = sum(b["checked"] - a["checked"] for a, b in zip(c0, c1))
    valid_all = sum(b["valid"] for b in c1)
    elapsed, (valid, checked) = multiseed.reduce_run(dist, elapsed, [valid, checked], args.red_dev)
    scratch, (valid_all,) = multiseed.reduce_run(dist, scratch, [valid_all], args.red_dev)
    digests = {}
    for i, e, c in zip(mine, engines, c1):
        st, par = e.read_tree(c["nodes"])
        digests[i] = multiseed.tree_digest(st, par)
    digests = multiseed.gather_digests(dist, digests)
    if rank != 0:
        return None
    summ, summ_path = pmc_summary(args.traffic, f"seeds{args.seeds}")
    geo = geometry(sc, env)
    e0 = engines[0]
    n_before = e0.counters()["nodes"]
    pmax = e0.info()["pmax"]
    scale = None
    if args.no_joint_nn:
        e0.collide_stats(True)
        e0.step(K, streams[0])
        torch.cuda.synchronize()
        cst = e0.collide_stats(False)
        per_launch = e0.kernel_times()
        nn_mode = e0.last_nn()
        kernels = dict(STAGE_KERNEL, nn_query=NN_KERNEL.get(nn_mode, "k_grid_nn1_runs"))
        if nn_mode == "tree":
            kernels["nn_build"] = "k_ct_dmerge"
        stages = stage_table(per_launch, cst, K, n_before, sc.dim, pmax, geo, nn_mode, kernels, summ)
        roof = roofline_of(stages, max(stages, key=lambda s: stages[s]["ms"]) if stages else None, cst, summ_path,
                           summ)
    else:
        # group 0: one round with the work counters on (each engine's own stages; summed over the
        # group), then one timed round: a joint round reports every stage (one launch per stage
        # for all the group's seeds, hipEvents on its joint stream), else the joint build + NN
        eg0, ss0, js0 = jgroups[0]
        for e in eg0:
            e.collide_stats(True)
        mpt.step_many(eg0, K, ss0, js0)
        torch.cuda.synchronize()
        csts = [e.collide_stats(False) for e in eg0]
        e0.enable_timing(True)
        mpt.step_many(eg0, K, ss0, js0)
        torch.cuda.synchronize()
        nj = len(eg0)
        agg = {k: sum(c[k] for c in csts) for k in csts[0]}
        n_tot = sum(e.counters()["nodes"] for e in eg0) - len(eg0) * K  # nodes before the timed call (upper bound)
        try:
            jst = mpt.joint_stage_times(js0)
        except mpt.MptError:
            jst = None
        if jst is not None:
            stages = joint_stage_table(jst, agg, K, nj, max(n_tot, 1), sc.dim, pmax, geo, summ)
            # event-free stage times (information only): a recorded round carries seven event
            # packets; when the stages sum to more than a timed round, scaled to it.  The rates
            # and fractions stay on the measured stage times -- the durations a kernel trace of
            # the same round shows (the committed profiles' steady_us), so they can be checked
            tot = sum(st["ms"] for st in stages.values())
            scale = min(1.0, (1e3 * elapsed / args.steps) / tot) if tot > 0 else 1.0
            for st in stages.values():
                st["ms_event_free"] = round(st["ms"] * scale, 4)
        else:
            try:
                jt = mpt.joint_times(js0)
            except mpt.MptError:
                jt = None  # no joint launch: every tree still below the Morton-tree size (small runs)
            per_launch = dict(e0.kernel_times())
            per_launch.pop("nn_query", None)
            per_launch.pop("nn_build", None)
            kernels = {s: k for s, k in STAGE_KERNEL.items() if s not in ("nn_query", "nn_build")}
            stages = stage_table(per_launch, csts[0], K, n_before, sc.dim, pmax, geo, "tree", kernels, summ)
            if jt:
                js = {"nn_build": jt["build"], "nn_query": jt["nn"]}
                stages.update(joint_stage_table(js, agg, K, nj, max(n_tot, 1), sc.dim, pmax, geo, summ))
        dom = "nn_query" if "nn_query" in stages else (max(stages, key=lambda k: stages[k]["ms"]) if stages else None)
        roof = roofline_of(stages, dom, dict(agg, seeds_in_group=nj), summ_path, summ)
        if scale is not None:
            roof["stage_time_scale"] = round(scale, 4)
        roof["round"] = round_roof(stages, 1e3 * elapsed / args.steps)
    import hashlib

    all_digest = hashlib.sha256("".join(digests[i] for i in sorted(digests)).encode()).hexdigest()
    n_local = len(mine)
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
                               f"grown from per-seed starts ({args.seed_start}), {K} extensions per seed per round",
                   "seeds": args.seeds, "seeds_per_gpu": n_local, "seed_base": args.seed,
                   "extensions_per_seed_round": K, "rounds_before_timing": args.warmup,
                   "streams_per_gpu": len(streams), "joint_nn": not args.no_joint_nn, "joint_groups": G,
                   "parallelism": f"seeds sharded over {world} GPU(s)"},
        "checked_per_s": checked / elapsed,
        "valid_fraction": valid / max(checked, 1),
        "per_seed_valid_per_s": valid / elapsed / max(args.seeds, 1),
        "host_enqueue_ms_per_step": 1e3 * host / args.steps,
        "seeds_digest": all_digest,
        "world_size": dist.get_world_size() if dist else 1,
        "from_scratch": {"rounds": args.warmup + args.steps, "wall_s": round(scratch, 4),
                         "valid_per_s": valid_all / scratch, "process_warmup_s": round(process_warmup, 4),
                         "note": "wall time of every round from the seeds' start states (the warm-up rounds, "
                                 "their first-use reservations, and the timed rounds), max over ranks, in a "
                                 "process whose HIP kernels and streams have run once (process_warmup_s: a "
                                 "throwaway two-engine round and the streams' first work, before the clock)"},
        "roofline": roof,
        "cpu_baseline": None,
    }


# ----------------------------------------------------------------------------- variants

# the secondary workloads measured in the same run as config 2 (one short leg each, in a
# process of its own so one leg's device state never affects another's timing): name ->
# (script, arguments).  The two config-5 legs run the same rounds (C5_STEPS, C5_WARMUP).
_C5 = ["--steps", str(C5_STEPS), "--warmup", str(C5_WARMUP)]
VARIANTS = {
    "blimp-room": ("bench.py", ["--workload", "blimp-room", "--steps", "20", "--warmup", "3"]),
    "snake": ("bench.py", ["--workload", "snake", "--steps", "10", "--warmup", "3"]),
    "seeds=32": ("bench.py", ["--seeds", "32"] + _C5),
    "seeds=256": ("bench.py", ["--seeds", "256"] + _C5),
    "prm": ("scripts/bench_prm.py", ["--reps", "3", "--bounds", "rooms"]),
    "distance": ("scripts/bench_distance.py", ["--steps", "10", "--warmup", "3"]),
}


def run_variants(detail=None):
    """Each leg's line (no CPU baseline, no nested legs), condensed: value, ms_per_step, the
    dominant stage's roofline, every stage's time and fractions, and (config 5) the seeds
    digest and from-scratch time; a leg that fails reports its error instead.  A bench.py leg
    writes its full line to a detail file of its own, which is what is condensed here."""
    out = {}
    ddir = os.path.dirname(detail) if detail else os.path.join(os.environ.get("TMPDIR", "/tmp"), f"mpt_{os.getpid()}")
    for name, (script, extra) in VARIANTS.items():
        cmd = [sys.executable, os.path.join(REPO, script), "--no-cpu"] + extra
        leg_detail = None
        if script == "bench.py":
            leg_detail = os.path.join(ddir, f"bench_detail_{name.replace('=', '')}.json")
            cmd += ["--no-variants", "--detail", leg_detail]
        t0 = time.perf_counter()
        try:
            p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=dict(os.environ))
            line = [x for x in p.stdout.splitlines() if x.startswith("{")]
            if p.returncode != 0 or not line:
                out[name] = {"error": f"rc={p.returncode}", "stderr_tail": p.stderr[-800:]}
                continue
            d = json.loads(line[-1])
            if leg_detail:
                try:
                    d = json.load(open(leg_detail))
                except (OSError, ValueError):
                    pass
        except subprocess.TimeoutExpired:
            out[name] = {"error": "timeout"}
            continue
        out[name] = condense(d)
        out[name]["leg_wall_s"] = round(time.perf_counter() - t0, 1)
    return out


# ----------------------------------------------------------------------------- the printed line

# The printed line stays well inside the driver's 8 KB stdout tail: every leg's value, time,
# dominant roofline and digest; the full stage tables go to the detail file (--detail).
ROOF_KEYS = ("bound", "achieved", "peak", "unit", "frac", "traffic", "traffic_over_compulsory", "frac_hbm_measured",
             "kernel", "stage", "ms_per_launch", "algorithmic_bytes", "pmc_source", "profile_us_per_launch",
             "frac_from_profile", "stage_time_scale")
LEG_ROOF_KEYS = ("bound", "achieved", "unit", "frac", "traffic_over_compulsory", "kernel", "ms_per_launch", "pmc_source",
                 "profile_us_per_launch", "frac_from_profile")


def compact_roof(roof, keys=ROOF_KEYS, stages_ms=True):
    r = {k: roof[k] for k in keys if roof.get(k) is not None}
    st = roof.get("stages") or {}
    if stages_ms and st:
        r["stages_ms"] = {s: v.get("ms_event_free", v.get("ms")) for s, v in st.items()}
    if roof.get("round"):
        r["round"] = roof["round"]
    return r


def compact_leg(leg):
    if "error" in leg:
        return {"error": leg["error"], "stderr_tail": (leg.get("stderr_tail") or "")[-300:]}
    out = {k: leg[k] for k in ("value", "unit", "ms_per_step", "wall_ms", "steps", "warmup", "valid_fraction",
                               "seeds_digest", "world_size", "leg_wall_s") if leg.get(k) is not None}
    if leg.get("from_scratch"):
        fs = leg["from_scratch"]
        out["from_scratch"] = {"rounds": fs.get("rounds"), "wall_s": fs.get("wall_s"),
                               "valid_per_s": fs.get("valid_per_s"), "process_warmup_s": fs.get("process_warmup_s")}
    cfg = leg.get("config") or {}
    for k in ("bounds", "free_fraction", "edges"):
        if k in cfg:
            out[k] = cfg[k]
    out["roofline"] = compact_roof(leg.get("roofline") or {}, LEG_ROOF_KEYS, stages_ms=False)
    return out


def compact_line(out, detail):
    line = {k: v for k, v in out.items() if k not in ("roofline", "variants", "config5", "config2", "cpu_baseline",
                                                       "kernel_ms_per_round", "from_scratch")}
    line["roofline"] = compact_roof(out.get("roofline") or {})
    if out.get("from_scratch"):
        fs = out["from_scratch"]
        line["from_scratch"] = {k: fs.get(k) for k in ("rounds", "wall_s", "valid_per_s", "process_warmup_s")}
    cb = out.get("cpu_baseline")
    if cb:
        line["cpu_baseline"] = {k: cb.get(k) for k in ("value", "unit", "cores", "kind", "sample", "cpu")}
        line["cpu_baseline"]["single_core"] = (cb.get("single_core") or {}).get("value")
        line["cpu_baseline"]["flann_rebuild_per_insert"] = (cb.get("flann_rebuild_per_insert") or {}).get("value")
    elif "cpu_baseline" in out:
        line["cpu_baseline"] = None
    if out.get("config2"):
        line["config2"] = compact_leg(out["config2"])
    if out.get("config5"):
        line["config5"] = {k: v for k, v in out["config5"].items() if k != "from_scratch"}
        fs = out["config5"].get("from_scratch") or {}
        line["config5"]["from_scratch_valid_per_s"] = fs.get("valid_per_s")
    if out.get("variants"):
        line["variants"] = {k: compact_leg(v) for k, v in out["variants"].items()}
    if detail:
        line["detail"] = os.path.relpath(detail, REPO) if detail.startswith(REPO) else detail
    return line


def condense(d):
    roof = d.get("roofline") or {}
    leg = {k: d.get(k) for k in ("metric", "value", "unit", "ms_per_step", "steps", "warmup", "valid_fraction",
                                 "scaling", "seeds_digest", "per_seed_valid_per_s", "host_enqueue_ms_per_step",
                                 "n_gpus", "world_size", "from_scratch", "edges_checked_per_s", "wall_ms",
                                 "device_ms", "work_per_step", "parity_sample_bitexact")
           if d.get(k) is not None}
    leg["config"] = d.get("config")
    leg["roofline"] = {k: roof.get(k) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel",
                                                "stage", "ms_per_launch", "pmc_source", "stage_time_scale",
                                                "profile_us_per_launch", "frac_from_profile",
                                                "frac_hbm_measured", "traffic_over_compulsory", "work")
                       if k in roof}
    leg["stages"] = {s: {k: v for k, v in st.items()
                         if k in ("ms", "ms_event_free", "frac_hbm_compulsory", "frac_hbm_measured",
                                  "traffic_over_compulsory", "frac_fp64", "kernel", "nn_points_per_query",
                                  "nn_boxes_per_query", "nn_steps_per_query")}
                     for s, st in (roof.get("stages") or {}).items()}
    return leg


def config5_summary(c5_256, c5_32=None):
    """The north-star scaling config in every line: the 256-seed run at this N (a leg of its
    own at N = 1, the in-world leg at N > 1), and at N = 1 the 32-seed leg one GPU of eight
    would run, at the same rounds: per-GPU ratio = v32 / v256, projected 8-GPU speed-up =
    8 x v32 / v256 (the driver's own N = 8 run measures it when it gets a node)."""
    if not c5_256 or "value" not in c5_256:
        return {"error": "config-5 leg missing", "leg": c5_256}
    out = {"seeds": (c5_256.get("config") or {}).get("seeds", 256), "value": c5_256["value"], "unit": c5_256.get("unit"), "ms_per_step": c5_256["ms_per_step"],
           "steps": c5_256["steps"], "warmup": c5_256["warmup"], "n_gpus": c5_256.get("n_gpus"),
           "world_size": c5_256.get("world_size"), "scaling": "strong", "seeds_digest": c5_256.get("seeds_digest"),
           "from_scratch": c5_256.get("from_scratch")}
    if c5_32 and "value" in c5_32:
        same = (c5_32["steps"], c5_32["warmup"]) == (c5_256["steps"], c5_256["warmup"])
        r = c5_32["value"] / c5_256["value"]
        out.update({"seeds32_value": c5_32["value"], "same_rounds": same, "per_gpu_ratio": round(r, 4),
                    "projected_8gpu_speedup": round(8 * r, 3)})
    return out


# The line's two scaling bases, the same keys at every N: `value` is config 2 (BASELINE configs[1],
# one 100k-node tree a rank: weak scaling, value(N) = N ranks' valid extensions / max-over-ranks
# time); `c5_*` is config 5 (BASELINE configs[4], the north star's scaling claim: 256 seeds
# sharded contiguously over the N ranks, strong scaling, the same trees -- c5_seeds_digest -- at
# every N).  At N = 1 c5_* is the seeds=256 leg, at N > 1 the leg run in the same world.
SCALING_BASIS = "value: config 2, a 100k tree a rank (weak); c5_*: config 5, 256 seeds over the ranks (strong)"


def c5_keys(leg):
    """The config-5 quantities under one key set at every N (see SCALING_BASIS)."""
    if not leg or "value" not in leg:
        return {"c5_value": None, "c5_error": (leg or {}).get("error", "config-5 leg missing")}
    return {"c5_value": leg["value"], "c5_ms_per_step": leg.get("ms_per_step"),
            "c5_seeds": (leg.get("config") or {}).get("seeds"), "c5_seeds_digest": leg.get("seeds_digest"),
            "c5_world_size": leg.get("world_size"), "c5_steps": leg.get("steps"), "c5_warmup": leg.get("warmup"),
            "c5_scaling": "strong"}


def attach_config5(out, c5_leg, variants=None):
    """The config-5 part of the line at any N: c5_* keys and the `config5` summary; at N = 1
    (variants: the legs run beside config 2) from the seeds=256 / seeds=32 legs, at N > 1
    from the in-world leg (c5_leg)."""
    if variants is not None:
        out["variants"] = variants
        c5_leg = variants.get("seeds=256")
        out["config5"] = config5_summary(c5_leg, variants.get("seeds=32"))
    else:
        out["config5"] = config5_summary(c5_leg)
        if isinstance((c5_leg or {}).get("roofline"), dict):
            out["config5"]["roofline"] = compact_roof(c5_leg["roofline"], LEG_ROOF_KEYS, stages_ms=False)
    out.update(c5_keys(c5_leg))
    out["scaling_basis"] = SCALING_BASIS
    return out


# ----------------------------------------------------------------------------- main

def free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n):
    """`bench.py --gpus N` without torchrun: the same command under torch.distributed.run with N
    ranks on this node (127.0.0.1), started as a child process -- nothing here has touched the
    GPU yet -- whose exit code is returned."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def main():
    args = parse()
    ws = os.environ.get("WORLD_SIZE")
    if ws is None and args.gpus is not None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    if ws is not None and args.gpus is not None and int(ws) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}")
    import torch

    world = int(ws or "1")
    args.gpus = world
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # MPT_DIST_BACKEND=gloo + MPT_BENCH_DEVICE=0: several ranks on one GPU (the multi-rank path
    # rehearsed on a one-GPU box, tests/test_bench_gpu.py); the driver's runs use RCCL, one
    # rank per GPU
    backend = os.environ.get("MPT_DIST_BACKEND", "nccl")
    if os.environ.get("MPT_BENCH_DEVICE") is not None:
        local = int(os.environ["MPT_BENCH_DEVICE"])
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    red_dev = "cuda" if backend == "nccl" else "cpu"
    args.red_dev = red_dev
    import motionplanningtoolkit_amd as mpt
    from motionplanningtoolkit_amd import multiseed, scenes

    mpt.init(local)
    torch.cuda.set_device(local)
    if args.seeds > 0:
        out = run_seeds(args, world, rank, dist, torch, mpt, multiseed, scenes)
    else:
        out = run_tree(args, world, rank, dist, torch, mpt, multiseed, scenes)
        if world > 1:
            # BASELINE config 5 in the same torchrun world: args.c5_seeds seeds sharded
            # contiguously over the ranks (32 per GPU at 8 GPUs), strong scaling; its seeds
            # digest equals the N = 1 run's (the seeds=256 leg) for the same rounds.  The top
            # level stays config 2 at every N (one basis for the driver's curve), config 5 goes
            # under the c5_* keys (SCALING_BASIS)
            a5 = argparse.Namespace(**vars(args))
            a5.seeds, a5.steps, a5.warmup = args.c5_seeds, args.c5_steps, args.c5_warmup
            c5 = run_seeds(a5, world, rank, dist, torch, mpt, multiseed, scenes)
            if out is not None:
                attach_config5(out, c5)
        elif out is not None and not args.no_variants and args.workload == "blimp":
            attach_config5(out, None, run_variants(args.detail))
    if out is not None:
        if args.detail:
            try:
                os.makedirs(os.path.dirname(args.detail), exist_ok=True)
                with open(args.detail, "w") as f:
                    json.dump(out, f, indent=1)
            except OSError:
                pass
        print(json.dumps(compact_line(out, args.detail)))
    if dist:
        dist.destroy_process_group()


def run_tree(args, world, rank, dist, torch, mpt, multiseed, scenes):
    """BASELINE config 2 (or --workload's variant): one tree of args.tree nodes per rank, reset
    to its base inside every timed round; returns the line on rank 0 (None elsewhere)."""
    stream = torch.cuda.current_stream()
    red_dev = args.red_dev
    if args.workload == "snake":
        sc = scenes.snake_scenario("corridor")
        workload = (f"snake.inst: snake_trailers ({sc.links} unit-box links, T=10) in the synthetic corridor "
                    f"({sc.env_tris.shape[0]} tris), batched RRT round over a {args.tree}-node tree")
    elif args.workload == "blimp-room":
        sc = scenes.blimp_room_scenario()
        workload = ("blimp.inst: blimp (1355 tris) vs single-room env (model.dae, 316 tris), tree and samples inside "
                    f"the room's box (collision-heavy variant), batched RRT round over a {args.tree}-node tree")
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

    elapsed, (valid, checked) = multiseed.reduce_run(dist, elapsed, [valid, checked], red_dev)

    if rank != 0:
        eng.close()
        return None

    steps = args.steps
    # hipEvents on the launch stream, recorded every n-th timed round into the engine's event
    # ring and read only now (no host sync inside the timed region)
    ktimes, kt_rounds = eng.kernel_times_sum()
    per_launch = {k: v / max(kt_rounds, 1) for k, v in ktimes.items()}
    # one more round, outside the timed region, with the collision work counters on
    eng.collide_stats(True)
    round_()
    cst = eng.collide_stats(False)
    nn_mode = eng.last_nn()
    d = sc.dim
    kernels = dict(STAGE_KERNEL, nn_query=NN_KERNEL.get(nn_mode, "k_grid_nn1_runs"))
    if nn_mode == "grid":  # the instantiation (its PMC row): queries bucketed by the grid count launch
        kernels["nn_query"] = f"k_grid_nn1_runs_sorted<{d},"
    if nn_mode == "tree":
        kernels["nn_build"] = "k_ct_dmerge"
    summ, summ_path = pmc_summary(args.traffic, args.workload)
    stages = stage_table(per_launch, cst, K, n0, d, eng.info()["pmax"], geometry(sc, env), nn_mode, kernels, summ)
    dominant = max(stages, key=lambda s: stages[s]["ms"]) if stages else None
    roof = roofline_of(stages, dominant, cst, summ_path, summ)
    roof["round"] = round_roof(stages, 1e3 * elapsed / steps)

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
        "world_size": dist.get_world_size() if dist else 1,
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
    eng.close()  # its device memory, before the next leg allocates
    return out


if __name__ == "__main__":
    main()
