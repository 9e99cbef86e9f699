#!/bin/bash
# Config 5: code plan folded into k_pt_bbox vs its own launch (interleaved repeats).
OUT=gpurun_out/ab5f; mkdir -p $OUT
for p in 0 1 0 1 0 1; do
  timeout -k 10 180 env MPT_PT_PLAN_LAUNCH=$p python bench.py --seeds 256 --steps 8 --warmup 3 --no-cpu > $OUT/p$p.log 2>&1 || exit $?
  grep '^{' $OUT/p$p.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('plan_launch', $p, round(d['value']/1e6,2), round(d['ms_per_step'],3), d['seeds_digest'][:16])"
done
echo done
