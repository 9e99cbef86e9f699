"""Where config 5's NN bytes come from: the joint NN launch (k_ct_nn1_jobs)
replayed alone after the bench's rounds, under different cache states, for rocprofv3's
FETCH_SIZE / WRITE_SIZE passes and a kernel trace.

  python scripts/nn_traffic.py [--seeds 256] [--rounds 30] [--out gpurun_out/nn_traffic.json]

Grows `seeds` wall-start blimp trees in one step_many group for `rounds` rounds of 4096
extensions (bench.py --seeds N's shape), then launches the last round's NN again
(mpt_rrt_joint_replay_nn: same jobs, same index, the same results rewritten), each replay
bracketed by hipEvents on the joint stream and separated by device syncs:

  replays (in dispatch order after the rounds' launches):
    after_round     right after the round (the round's last kernels: collide, append)
    after_writes    after writing 512 MiB (dirty lines of another buffer in L2 / MALL: their
                    write-back lands in whichever kernel evicts them)
    pP_flush        XCD mapping P (mpt_rrt_joint_replay_nn parts: 0 = every tree over all eight
                    XCDs, P > 0 = each tree in P runs, one XCD each) after reading a 2 GiB buffer
                    twice (L2 and the 256 MiB MALL hold clean, unrelated lines)
    pP_b2b          the same launch again at once

The ids and squared distances of the round are read before and after: identical.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def labels(seeds):
    out = ["after_round", "after_writes"]
    for p in (0, 1, 2, 4, 8):
        if seeds * p % 8 == 0 and 4096 % max(p, 1) == 0:
            out += [f"p{p}_flush", f"p{p}_b2b"]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=30)
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "nn_traffic.json"))
    args = ap.parse_args()
    import torch

    import bench
    import motionplanningtoolkit_amd as mpt
    from motionplanningtoolkit_amd import scenes

    mpt.init(0)
    sc = scenes.blimp_scenario("all")
    env = mpt.Environment(sc.env_tris, sc.env_tf)
    ag = mpt.AgentMesh(sc.agent_tris)
    K, base = 4096, 1000
    engs = []
    for i in range(args.seeds):
        e = mpt.RRTEngine(env, ag, sc.kind, sc.prm, sc.ranges, sc.steer_dt, sc.cc_dt, 1 + args.rounds * K, base + i)
        e.add_nodes(bench.seed_start(base + i, env, ag, mpt, "walls"))
        e.set_nn("auto")
        engs.append(e)
    joint = torch.cuda.Stream()
    t0 = time.perf_counter()
    for r in range(args.rounds):
        mpt.step_many(engs, K, [joint] * len(engs), joint)
        if r % 5 == 4:
            torch.cuda.synchronize()
            print(f"round {r + 1}: {time.perf_counter() - t0:.1f} s", flush=True)
    torch.cuda.synchronize()
    nodes = sum(e.counters()["nodes"] for e in engs) - len(engs) * K  # indexed in the last round
    pick = [0, len(engs) // 2, len(engs) - 1]
    before = [engs[i].last_round(K)[1] for i in pick]
    flush = torch.empty(1 << 29, dtype=torch.float32, device="cuda")  # 2 GiB
    flush.fill_(1.0)
    dirty = torch.empty(1 << 27, dtype=torch.float32, device="cuda")  # 512 MiB
    torch.cuda.synchronize()

    def do_flush():
        for _ in range(2):
            float(flush.sum())

    res = {}
    LABELS = labels(len(engs))
    for label in LABELS:
        if label.endswith("_flush"):
            do_flush()
        elif label == "after_writes":
            dirty.fill_(2.0)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(joint)
        mpt.joint_replay_nn(joint, parts=int(label[1:label.index("_")]) if label[0] == "p" else 0)
        b.record(joint)
        torch.cuda.synchronize()
        res[label] = round(a.elapsed_time(b), 4)
    after = [engs[i].last_round(K)[1] for i in pick]
    same = all(np.array_equal(x, y) for x, y in zip(before, after))
    out = {"seeds": args.seeds, "rounds": args.rounds, "queries": args.seeds * K, "nodes_indexed": int(nodes),
           "replay_ms": res, "replays_in_dispatch_order": LABELS, "ids_unchanged": same}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(out, open(args.out, "w"), indent=1)
    print(json.dumps(out))
    for e in engs:
        e.close()
    mpt.joint_release(joint)
    if not same:
        sys.exit("replayed NN ids differ")


if __name__ == "__main__":
    main()
