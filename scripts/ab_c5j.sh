#!/bin/bash
# Config 5 joint build: points per k_pt_bbox_jobs workgroup A/B (interleaved repeats).
OUT=gpurun_out/ab5j; mkdir -p $OUT
for p in 2048 8192 32768 2048 8192 32768; do
  timeout -k 10 180 env MPT_PT_BBOX_PTS=$p python bench.py --seeds 256 --steps 6 --warmup 3 --no-cpu > $OUT/p$p.log 2>&1 || exit $?
  grep '^{' $OUT/p$p.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('pts', $p, round(d['value']/1e6,2), round(d['ms_per_step'],3), d['seeds_digest'][:16])"
done
echo done
