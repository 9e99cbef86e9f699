"""Config 5's host enqueue against the GPU: after warm rounds, enqueue N joint rounds without a
sync (the time until the last step_many returns), then the wall time until they finish, and
each step_many call's own host time.  If the enqueue time approaches the wall time the rounds
wait on the host, not on the kernels.

  python scripts/c5_host_rate.py [--seeds 32] [--rounds 20]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--warm", type=int, default=5)
    a = ap.parse_args()
    import torch

    import bench
    import motionplanningtoolkit_amd as mpt
    from motionplanningtoolkit_amd import scenes

    mpt.init(0)
    sc = scenes.blimp_scenario("all")
    env = mpt.Environment(sc.env_tris, sc.env_tf)
    agent = mpt.AgentMesh(sc.agent_tris)
    K = 4096
    engines = []
    for i in range(a.seeds):
        e = mpt.RRTEngine(env, agent, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt,
                          1 + (a.rounds + a.warm + 2) * K, 1000 + i)
        e.add_nodes(bench.seed_start(1000 + i, env, agent, mpt, "walls"))
        e.set_nn("auto")
        engines.append(e)
    js = torch.cuda.Stream()
    for _ in range(a.warm):
        mpt.step_many(engines, K, [js] * len(engines), js)
    torch.cuda.synchronize()
    calls = []
    t0 = time.perf_counter()
    for _ in range(a.rounds):
        h = time.perf_counter()
        mpt.step_many(engines, K, [js] * len(engines), js)
        calls.append(time.perf_counter() - h)
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(json.dumps({"seeds": a.seeds, "rounds": a.rounds, "enqueue_ms_per_round": 1e3 * t_enq / a.rounds,
                      "wall_ms_per_round": 1e3 * t_all / a.rounds,
                      "call_ms": [round(1e3 * c, 3) for c in calls]}))
    for e in engines:
        e.close()
    mpt.joint_release(js)


if __name__ == "__main__":
    main()
