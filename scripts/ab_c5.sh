#!/bin/bash
# Config 5 (256 seeds): host launch threads x hardware queues A/B (one MI355X).
OUT=gpurun_out/ab5; mkdir -p $OUT
B="python bench.py --seeds 256 --steps 8 --warmup 3 --no-cpu"
for q in 4 16; do
  for t in 1 4 8; do
    timeout -k 10 180 env GPU_MAX_HW_QUEUES=$q $B --launch-threads $t > $OUT/q${q}_t$t.log 2>&1 || exit $?
    grep '^{' $OUT/q${q}_t$t.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('q', $q, 't', $t, round(d['value']/1e6,2), round(d['ms_per_step'],3), d['seeds_digest'][:16])"
  done
done
echo done
