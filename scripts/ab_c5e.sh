#!/bin/bash
# Config 5: joint-launch groups A/B (repeats for run-to-run spread).
OUT=gpurun_out/ab5e; mkdir -p $OUT
for g in 1 2 4 1 2 4; do
  timeout -k 10 180 python bench.py --seeds 256 --steps 8 --warmup 3 --no-cpu --joint-groups $g > $OUT/g$g.log 2>&1 || exit $?
  grep '^{' $OUT/g$g.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('groups', $g, round(d['value']/1e6,2), round(d['ms_per_step'],3), d['seeds_digest'][:16])"
done
echo done
