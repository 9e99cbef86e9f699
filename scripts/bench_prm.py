"""BASELINE config 4: PRM construction with radius neighbours over a ~200k-triangle env.

Workload: synthetic env = 25 x 25 copies of the model.dae room (197 500 triangles; the
reference's apartment.dae is missing), blimp agent (all 1355 triangles of blimp.3ds),
N milestones ~ U(Blimp::getStateVarRanges) with x, y, z over the whole multi-room extent
(--bounds rooms, the default; --bounds blimp: blimp.inst's [-100, 100]^3), radius chosen for a
mean of ~10 neighbours per milestone (counting both directions), cc_dt 0.1 (blimp.inst).  One call
of mpt_prm_connect: point-tree radius search, edge poses, batched collision, components.
Prints one JSON line: milestones/s, edges checked/s, per-stage device ms, and the oracle's
single-core rate on a bounded sample of the same roadmap (its first milestones).

  python scripts/bench_prm.py [--n 100000] [--reps 3]
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
HBM_PEAK_GBS = 8000.0


def latest_pmc(sub):
    """The newest committed rocprofv3 PMC summary of this workload (profiles/r*/<sub>/)."""
    import glob

    c = sorted(glob.glob(os.path.join(REPO, "profiles", "r[0-9][0-9]", sub, "pmc_summary.json")))
    return c[-1] if c else ""


def sweep_roofline(w, ms, n_agent, n_env, n_milestones, traffic_path):
    """The config-4 collision stage (sweep.hip: k_sweep_cands, k_sweep_sat, k_sweep_prm twice --
    one wave per edge over the agent's clusters, the edge's poses generated in the kernels from
    its two milestones, prm_edges.h): FP64 by SURVEY §8(d)'s model -- 750 flops per exact
    triangle test, 27 per (pair, pose) gate (the translated triangle's box and the overlap
    test), 45 per agent triangle rotated once per wave (R Q, 64 lanes) -- and HBM: compulsory =
    every input once -- the edges (source, target id, verdict byte), the milestones' keys and
    yaw (40 B), the agent triangles, the env tree's items and triangle records -- measured = the
    stage's rocprofv3 PMC traffic (every k_sweep* launch of one mpt_prm_connect call)."""
    t = ms * 1e-3
    flops = 750.0 * w["sat_tests"] + 27.0 * w["gate_tests"] + 45.0 * 64 * w["waves"]
    items = n_env + -(-n_env // 8)
    comp = w["edges"] * 9 + n_milestones * 40 + n_agent * 72 + items * 32 + n_env * 384
    out = {"bound": "fp64_valu", "kernel": "k_sweep_cands + k_sweep_sat + k_sweep_prm",
           "achieved": round(flops / t / 1e12, 3), "peak": FP64_PEAK_TFLOPS,
           "unit": "TFLOP/s", "frac": round(flops / t / 1e12 / FP64_PEAK_TFLOPS, 4),
           "note": "FP64 VALU roof (FCL's scalar operation order; no MFMA)",
           "compulsory_bytes": int(comp), "compulsory_gbs": round(comp / t / 1e9, 1),
           "frac_hbm_compulsory": round(comp / t / 1e9 / HBM_PEAK_GBS, 4), "ms_per_launch": round(ms, 4),
           "work": w, "traffic": None}
    path = traffic_path or latest_pmc("prm")
    try:
        summ = json.load(open(path))
        parts = [v["hbm_bytes_per_launch"] * v.get("launches", 1) for k, v in summ.items() if "k_sweep" in k]
        if not parts:
            raise StopIteration
        tr = sum(parts)
        # the stage's kernel time in the same profile (steady_us: the timed call's launches)
        prof_us = sum(v["steady_us"] * v.get("steady_launches", 1) for k, v in summ.items()
                      if "k_sweep" in k and v.get("steady_us"))
        if prof_us > 0:
            out["profile_us_per_launch"] = round(prof_us, 3)
        out.update({"traffic": int(tr), "traffic_gbs": round(tr / t / 1e9, 1),
                    "frac_hbm_measured": round(tr / t / 1e9 / HBM_PEAK_GBS, 4),
                    "traffic_over_compulsory": round(tr / comp, 2), "pmc_source": os.path.relpath(path, REPO)})
    except (OSError, ValueError, StopIteration):
        pass
    if out["frac"] < max(out["frac_hbm_compulsory"], out.get("frac_hbm_measured") or 0.0):
        out.update({"bound": "hbm", "achieved": out["compulsory_gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": out["frac_hbm_compulsory"]})
    if out.get("profile_us_per_launch"):
        # the same fraction on the profile's own kernel time (the line's is the stage's hipEvents)
        out["frac_from_profile"] = round(out["frac"] * ms * 1e3 / out["profile_us_per_launch"], 4)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--degree", type=float, default=10.0)
    ap.add_argument("--rooms", type=int, default=25)
    ap.add_argument("--cpu-n", type=int, default=3000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--traffic", default=None,
                    help="pmc_summary.json with k_sweep's traffic (default: the newest profiles/r*/prm/)")
    ap.add_argument("--collide", default="split", choices=["split", "fused"])
    ap.add_argument("--bounds", default="rooms", choices=["blimp", "rooms"],
                    help="milestone x, y, z: the whole multi-room extent (default: every room's walls in play, "
                         "tests/test_scale_gpu.py test_config4_rooms_at_size) or blimp.inst's [-100, 100]^3 (one "
                         "corner of the rooms)")
    a = ap.parse_args()

    import motionplanningtoolkit_amd as mpt
    from motionplanningtoolkit_amd import scenes

    mpt.init(0)
    mpt.set_collide_mode(a.collide)
    sc = scenes.blimp_scenario("all")
    env_t = scenes.rooms_env(a.rooms, a.rooms)
    env, ag = mpt.Environment(env_t, sc.env_tf), mpt.AgentMesh(sc.agent_tris)
    rng = np.random.default_rng(0)
    st = rng.uniform(sc.ranges[:, 0], sc.ranges[:, 1], size=(a.n, sc.dim))
    lo, hi = sc.ranges[:3, 0], sc.ranges[:3, 1]
    if a.bounds == "rooms":
        lo, hi = env_t.reshape(-1, 3).min(0), env_t.reshape(-1, 3).max(0)
        st[:, :3] = rng.uniform(lo, hi, size=(a.n, 3))
    vol = float(np.prod(hi - lo))
    r = (a.degree * vol / (a.n * 4.0 / 3.0 * math.pi)) ** (1.0 / 3.0)
    r2 = r * r
    mpt.prm_connect(env, ag, 1, st[: min(a.n, 2000)], r2, sc.cc_dt)  # warm-up (allocations)
    # one call with the sweep's work counters on (an atomic per wave: untimed), before the timed
    # calls, so that a profile's last call (scripts/profile_all.sh: last:k_sort_segments) is timed
    mpt.prm_stats(True)
    mpt.prm_connect(env, ag, 1, st, r2, sc.cc_dt)
    work = mpt.prm_stats(False)
    walls, res = [], None
    for _ in range(a.reps):
        t0 = time.perf_counter()
        res = mpt.prm_connect(env, ag, 1, st, r2, sc.cc_dt)
        walls.append(time.perf_counter() - t0)
    E = len(res["edges"])
    ms = res["ms"]
    wall = min(walls)
    roof = sweep_roofline(work, ms["collision"], len(sc.agent_tris), int(env.info()["triangles"]), a.n, a.traffic)
    out = {
        "metric": "PRM roadmap construction (radius neighbours + edge collision checks), config 4",
        "value": a.n / wall, "unit": "milestones/s", "edges_checked_per_s": E / wall,
        "wall_ms": 1e3 * wall, "device_ms": ms, "dtype": "f64", "data": "synthetic milestones",
        "config": {"workload": f"blimp ({len(sc.agent_tris)} tris) PRM in {a.rooms}x{a.rooms} rooms "
                               f"({len(env_t)} tris)", "milestones": a.n, "radius": r, "edges": E,
                   "free_fraction": float(1.0 - res["verdict"].mean()) if E else None,
                   "components": int(len(np.unique(res["comp"]))), "collide_mode": a.collide,
                   "bounds": a.bounds},
        "roofline": roof,
    }
    if not a.no_cpu:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle as orc

        k = min(a.cpu_n, a.n)
        bvh = orc.BVH(env_t)
        t0 = time.perf_counter()
        e_ref, v_ref, _ = orc.prm_radius(bvh, sc.env_tf, sc.agent_tris, st[:k], r2, sc.cc_dt, nthreads=1)
        dt = time.perf_counter() - t0
        sub = mpt.prm_connect(env, ag, 1, st[:k], r2, sc.cc_dt)
        out["cpu_baseline"] = {"value": len(e_ref) / dt, "unit": "edges checked/s", "cores": 1, "kind": "port",
                               "sample": f"the roadmap of the first {k} milestones ({len(e_ref)} edges), "
                                         f"oracle/mpt_oracle.c orc_prm_radius, {dt:.1f} s"}
        out["parity_sample"] = bool(np.array_equal(sub["edges"], e_ref) and np.array_equal(sub["verdict"], v_ref))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
