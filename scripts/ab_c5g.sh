#!/bin/bash
# Config 5 with the joint NN launch: hardware queues per process (HIP default 4) A/B.
OUT=gpurun_out/ab5g; mkdir -p $OUT
for q in 4 8 16 4 8 16; do
  timeout -k 10 180 env GPU_MAX_HW_QUEUES=$q python bench.py --seeds 256 --steps 6 --warmup 3 --no-cpu > $OUT/q$q.log 2>&1 || exit $?
  grep '^{' $OUT/q$q.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('queues', $q, round(d['value']/1e6,2), round(d['ms_per_step'],3), d['seeds_digest'][:16])"
done
echo done
