"""Host-side enqueue rate of config-2 rounds vs the GPU's: time to enqueue N rounds (no
sync) and the wall time until they finish.  If the first approaches the second, rounds are
bound by the host's launch path, not by the kernels.
Usage: python scripts/host_rate.py [--rounds 100]"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=100)
    ap.add_argument("--workload", default="blimp", choices=["blimp", "blimp-room"])
    a = ap.parse_args()
    import torch
    import motionplanningtoolkit_amd as mpt
    from motionplanningtoolkit_amd import scenes
    torch.cuda.init()
    mpt.init(0)
    sc = scenes.blimp_scenario("all") if a.workload == "blimp" else scenes.blimp_room_scenario()
    n0, K = 100_000, 65_536
    tree = np.random.default_rng(1000).uniform(sc.ranges[:, 0], sc.ranges[:, 1], size=(n0, sc.dim))
    eng = mpt.RRTEngine(mpt.Environment(sc.env_tris, sc.env_tf), mpt.AgentMesh(sc.agent_tris), sc.kind, sc.prm,
                        sc.ranges, sc.steer_dt, sc.cc_dt, n0 + K, 1000)
    eng.add_nodes(tree)
    eng.set_nn("auto")
    eng.enable_timing(False)
    stream = torch.cuda.current_stream()
    for _ in range(5):
        eng.set_size(n0, stream)
        eng.step(K, stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.rounds):
        eng.set_size(n0, stream)
        eng.step(K, stream)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"enqueue {1e6 * (t1 - t0) / a.rounds:.1f} us/round, wall {1e6 * (t2 - t0) / a.rounds:.1f} us/round "
          f"({a.rounds} rounds)", flush=True)


if __name__ == "__main__":
    main()
