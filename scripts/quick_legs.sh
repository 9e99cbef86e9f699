#!/bin/bash
# Usage: TAG=x bash scripts/quick_legs.sh -- config 2, the room and the snake (bench lines,
# twice each for config 2 and the room) into gpurun_out/$TAG/, then a summary
TAG=${TAG:?set TAG}
O=gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu --no-variants > $O/c2_$rep.json || exit 1
  timeout -k 10 120 python bench.py --workload blimp-room --steps 30 --warmup 5 --no-cpu --no-variants > $O/room_$rep.json || exit 1
done
timeout -k 10 120 python bench.py --workload snake --steps 10 --warmup 3 --no-cpu --no-variants > $O/snake.json || exit 1
python - $O <<'PY'
import json, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(f.split("/")[-1], round(d["value"] / 1e6, 1), round(d["ms_per_step"], 4))
    except Exception:
        pass
PY
