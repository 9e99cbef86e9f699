"""Config 5 from the seeds' start states: wall time of each of the first rounds (synchronised
after each), to see what a planner run pays before its steady state (bench.py from_scratch).

  python scripts/scratch_rounds.py [--seeds 32] [--rounds 8]
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
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--warm", default="none", choices=["none", "stream", "group"],
                    help="before the timed rounds: nothing; a torch op on the joint stream; or also a throwaway "
                         "two-engine group's round (every kernel of a joint round launched once in the process)")
    a = ap.parse_args()
    import torch

    import bench
    import motionplanningtoolkit_amd as mpt
    from motionplanningtoolkit_amd import scenes

    mpt.init(0)
    sc = scenes.blimp_scenario("all")
    env = mpt.Environment(sc.env_tris, sc.env_tf)
    agent = mpt.AgentMesh(sc.agent_tris)
    K = a.batch
    t0 = time.perf_counter()
    engines = []
    for i in range(a.seeds):
        e = mpt.RRTEngine(env, agent, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, 1 + (a.rounds + 2) * K,
                          1000 + i)
        e.add_nodes(bench.seed_start(1000 + i, env, agent, mpt, "walls"))
        e.set_nn("auto")
        engines.append(e)
    torch.cuda.synchronize()
    setup = time.perf_counter() - t0
    js = torch.cuda.Stream()
    if a.warm != "none":
        with torch.cuda.stream(js):
            torch.zeros(1, device="cuda").add_(1)
    if a.warm == "group":
        tmp = []
        for i in range(2):
            e = mpt.RRTEngine(env, agent, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, 1 + 2 * K, 99 + i)
            e.add_nodes(bench.seed_start(1000 + i, env, agent, mpt, "walls"))
            e.set_nn("auto")
            tmp.append(e)
        ws = torch.cuda.Stream()
        mpt.step_many(tmp, K, [ws] * 2, ws)
        torch.cuda.synchronize()
        for e in tmp:
            e.close()
        mpt.joint_release(ws)
    ms = []
    for r in range(a.rounds):
        t = time.perf_counter()
        mpt.step_many(engines, K, [js] * len(engines), js)
        torch.cuda.synchronize()
        ms.append(round(1e3 * (time.perf_counter() - t), 3))
    print(json.dumps({"seeds": a.seeds, "warm": a.warm, "setup_s": round(setup, 3), "round_ms": ms}))


if __name__ == "__main__":
    main()
