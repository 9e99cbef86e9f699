"""Per-round view of a rocprofv3 kernel trace of bench.py (scripts/profile.sh, `kt` pass).

Rounds end at the engine's k_append_commit launch (grid rounds start with the grid count
launch, which also generates the samples; tree rounds with k_sample).  For the timed rounds (after
`--warmup`, `--steps` of them; the bench's extra untimed stats round is dropped) it prints
each kernel's mean / median duration, the kernels' busy time per round and the round span
(k_sample start to the next round's k_sample start), so the idle gaps between launches show.
With --json it writes the same numbers as profiles/<tag>/timed_rounds.json: the per-launch
averages over the timed region that bench.py's hipEvent stage times are compared with.

Usage: python scripts/trace_rounds.py gpurun_out/prof_r05/kt/run_kernel_trace.csv --warmup 3 --steps 20 [--json out]
"""
import argparse
import collections
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    rounds, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        if cur is None:
            cur = []
            rounds.append(cur)
        cur.append((name, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        if "k_append_commit" in name:
            cur = None
    if rounds and not any("k_append_commit" in n for n, _, _ in rounds[-1]):
        rounds.pop()  # trailing kernels after the last round
    timed = rounds[a.warmup:a.warmup + a.steps]
    per = collections.defaultdict(list)
    busy, span = [], []
    for i, rd in enumerate(timed):
        busy.append(sum(e - s for _, s, e in rd))
        nxt = rounds[a.warmup + i + 1][0][1] if a.warmup + i + 1 < len(rounds) else rd[-1][2]
        span.append(nxt - rd[0][1])
        for name, s, e in rd:
            per[name].append(e - s)
    out = {"rounds": len(timed), "busy_us_per_round": statistics.mean(busy) / 1e3,
           "span_us_per_round": statistics.mean(span) / 1e3, "kernels": {}}
    for name, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
        out["kernels"][short] = {"launches_per_round": len(v) / len(timed), "mean_us": statistics.mean(v) / 1e3,
                                 "median_us": statistics.median(v) / 1e3}
    print(f"timed rounds {out['rounds']}: busy {out['busy_us_per_round']:.1f} us, span {out['span_us_per_round']:.1f} us")
    for k, v in out["kernels"].items():
        print(f"  {k:60s} x{v['launches_per_round']:.2f} mean {v['mean_us']:8.2f} median {v['median_us']:8.2f}")
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
