#!/bin/bash
# Usage: TAG=x bash scripts/ab_legs.sh [legs...] -- bench legs for an A/B step, each under its own
# time limit, lines into gpurun_out/$TAG/<leg>.json and a one-line-per-leg summary.
# legs: c2 room snake c5_32 c5_256 distance prm (default: all)
TAG=${TAG:?set TAG}
O=gpurun_out/$TAG; mkdir -p $O
LEGS=("$@"); [ ${#LEGS[@]} -eq 0 ] && LEGS=(c2 room snake c5_32 c5_256 distance prm)
for leg in "${LEGS[@]}"; do
  case $leg in
    c2) cmd=(python bench.py --steps 30 --warmup 5 --no-cpu --no-variants --detail $O/c2_detail.json) ;;
    room) cmd=(python bench.py --workload blimp-room --steps 30 --warmup 5 --no-cpu --no-variants --detail $O/room_detail.json) ;;
    snake) cmd=(python bench.py --workload snake --steps 10 --warmup 3 --no-cpu --no-variants --detail $O/snake_detail.json) ;;
    c5_32) cmd=(python bench.py --seeds 32 --steps 25 --warmup 5 --no-cpu --detail $O/c5_32_detail.json) ;;
    c5_256) cmd=(python bench.py --seeds 256 --steps 25 --warmup 5 --no-cpu --detail $O/c5_256_detail.json) ;;
    distance) cmd=(python scripts/bench_distance.py --steps 10 --warmup 3 --no-cpu) ;;
    prm) cmd=(python scripts/bench_prm.py --reps 3 --bounds rooms --no-cpu) ;;
    *) echo "unknown leg $leg"; exit 2 ;;
  esac
  timeout -k 10 300 "${cmd[@]}" > $O/$leg.json 2> $O/$leg.err || { echo "$leg failed rc=$?"; tail -5 $O/$leg.err; exit 1; }
  echo "$leg done"
done
python - $O <<'PY'
import json, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    if f.endswith("_detail.json"):
        continue
    try:
        d = json.loads([l for l in open(f).read().splitlines() if l.startswith("{")][-1])
        r = d.get("roofline") or {}
        print(f.split("/")[-1], round(d["value"] / 1e6, 3), d.get("unit"), round(d.get("ms_per_step") or d.get("device_ms") or 0, 4),
              d.get("seeds_digest", "")[:8], r.get("kernel"), r.get("ms_per_launch"), r.get("frac"))
    except Exception as e:
        print(f, "unparsed", e)
PY
