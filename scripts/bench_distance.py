"""Mesh-vs-mesh distance throughput (no reference caller, so no baseline
number): blimp (blimp.3ds, all 1355 triangles by default) at N random poses in and around the
single-room env (model.dae, 316 triangles), one pose per edge, one mpt_distance_batch_device
call per step with inputs resident in HBM.  Prints one JSON line: poses/s, the kernel's
hipEvent time, work counters and the oracle's single-core rate on a bounded sample.

  python scripts/bench_distance.py [--n 65536] [--steps 10] [--agent all|last]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

FP64_PEAK_TFLOPS = 78.6
TRI_DISTANCE_FLOPS = 700  # FP64 ops of one triDistance call: 9 segPoints (~60) + tests


def blimp_poses(rng, n):
    """Poses as Blimp::stateToFCLTransform makes them (rotation about z), spread over the
    room's box and a margin around it."""
    t = rng.uniform([-30, -30, -30], [207, 168, 144], size=(n, 3))
    th = rng.uniform(0, 2 * math.pi, n)
    c, s = np.cos(th), np.sin(th)
    P = np.zeros((n, 12))
    P[:, 0], P[:, 1], P[:, 3], P[:, 4], P[:, 8] = c, s, -s, c, 1.0
    P[:, 9:] = t
    return P


HBM_PEAK_GBS = 8000.0


def distance_roofline(out, a, n_agent, n_env, ms):
    """k_distance: FP64 (TRI_DISTANCE_FLOPS per triDistance call) against the FP64 VALU roof;
    compulsory HBM bytes = the poses (96 B), the edge offsets, the results, the agent
    triangles (72 B) and the env records (384 B a triangle + 32 B a tree item) once; measured
    traffic from the newest committed PMC summary (profiles/r*/distance/)."""
    import glob

    t = ms * 1e-3
    comp = a.n * (96 + 8 + 8) + n_agent * 72 + n_env * (384 + 32)
    roof = {"bound": "fp64_valu", "kernel": "k_distance", "achieved": round(out["fp64"]["achieved_tflops"], 3),
            "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(out["fp64"]["frac"], 4),
            "note": "FP64 VALU roof (FCL's scalar operation order; no MFMA)", "ms_per_launch": round(ms, 4),
            "compulsory_bytes": int(comp), "frac_hbm_compulsory": round(comp / t / 1e9 / HBM_PEAK_GBS, 4),
            "traffic": None, "work": out["work_per_step"]}
    c = sorted(glob.glob(os.path.join(REPO, "profiles", "r[0-9][0-9]", "distance", "pmc_summary.json")))
    if c:
        try:
            summ = json.load(open(c[-1]))
            kd = next(v for k, v in summ.items() if "k_distance" in k)
            tr = kd["hbm_bytes_per_launch"]
            roof.update({"traffic": int(tr), "frac_hbm_measured": round(tr / t / 1e9 / HBM_PEAK_GBS, 4),
                         "traffic_over_compulsory": round(tr / comp, 2), "pmc_source": os.path.relpath(c[-1], REPO)})
            if kd.get("steady_us"):
                # the same fraction on the profile's own steady-state launch time
                roof.update({"profile_us_per_launch": kd["steady_us"],
                             "frac_from_profile": round(roof["frac"] * ms * 1e3 / kd["steady_us"], 4)})
        except (OSError, ValueError, StopIteration):
            pass
    return roof


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--agent", default="all", choices=["all", "last"])
    ap.add_argument("--cpu-poses", type=int, default=200)
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()

    import torch

    import motionplanningtoolkit_amd as mpt
    from motionplanningtoolkit_amd import scenes

    mpt.init(0)
    env_t = scenes.read_obj(scenes.mesh_path("env_model"))
    agent_t = scenes.read_obj(scenes.mesh_path("agent_blimp"), a.agent)
    env, ag = mpt.Environment(env_t), mpt.AgentMesh(agent_t)
    rng = np.random.default_rng(0)
    P = blimp_poses(rng, a.n)
    dev = torch.device("cuda", 0)
    d_poses = torch.from_numpy(P).to(dev)
    d_off = torch.arange(a.n + 1, dtype=torch.int64, device=dev)
    d_out = torch.empty(a.n, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream()

    def step():
        mpt.distance_batch_device(env, [ag], d_poses.data_ptr(), d_off.data_ptr(), a.n, a.n, d_out.data_ptr(), stream)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(a.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ms = ev0.elapsed_time(ev1) / a.steps

    mpt.set_collide_stats(True)
    step()
    st = mpt.last_collide_stats()
    mpt.set_collide_stats(False)
    waves, items, calls, pairs = st["units"], st["clusters"], st["node_visits"], st["tri_tests"]
    d = d_out.cpu().numpy()

    out = {
        "metric": "mesh-mesh distance queries/s (blimp vs single room)",
        "value": a.n / (ms * 1e-3), "unit": "poses/s", "ms_per_step": ms, "steps": a.steps,
        "wall_s": wall, "dtype": "f64", "data": "synthetic poses",
        "config": {"workload": f"blimp({len(agent_t)} tris) vs model.dae({len(env_t)} tris)", "poses": a.n},
        "work_per_step": {"clusters_walked": waves, "env_box_tests": items, "tri_distance_calls": calls,
                          "pair_box_tests": pairs},
        "fp64": {"flops_per_step": calls * TRI_DISTANCE_FLOPS,
                 "achieved_tflops": calls * TRI_DISTANCE_FLOPS / (ms * 1e-3) / 1e12,
                 "peak_tflops": FP64_PEAK_TFLOPS},
        "contact_fraction": float((d == 0).mean()),
    }
    out["fp64"]["frac"] = out["fp64"]["achieved_tflops"] / FP64_PEAK_TFLOPS
    out["roofline"] = distance_roofline(out, a, len(agent_t), len(env_t), ms)
    if not a.no_cpu:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle as orc

        k = min(a.cpu_poses, a.n)
        t0 = time.perf_counter()
        ref = orc.distance_batch(env_t, np.r_[np.eye(3).ravel(), 0, 0, 0], [agent_t], P[:k].reshape(-1, 1, 12),
                                 np.arange(k + 1), nthreads=1)
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": k / dt, "unit": "poses/s", "cores": 1, "kind": "port",
                               "sample": f"first {k} poses, oracle all-pairs with box-gap pruning"}
        out["parity_sample_bitexact"] = bool(np.array_equal(ref.view(np.uint64), d[:k].view(np.uint64)))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
