"""Print one line per bench log: value, ms/step, per-stage ms (helper for A/B runs)."""
import json
import sys

for f in sys.argv[1:]:
    try:
        line = [l for l in open(f) if l.startswith("{")][-1]
    except (IndexError, OSError):
        print(f, "no result")
        continue
    d = json.loads(line)
    k = d.get("kernel_ms_per_round", {})
    r = d["roofline"]
    w = r.get("work_per_round", {})
    print(f"{f.split('/')[-1]:18s} {d['value'] / 1e6:8.2f}M ms={d['ms_per_step']:.4f} "
          + " ".join(f"{s}={k[s]:.4f}" for s in ("sample", "nn_build", "nn_query", "steer", "collide", "append") if s in k)
          + f" | {r['kernel']} {r['ms_per_launch']} frac={r['frac']} pts={w.get('nn_points')}")
