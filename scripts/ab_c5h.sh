#!/bin/bash
# Config 5 with the joint NN launch: engine streams A/B (4 hardware queues).
OUT=gpurun_out/ab5h; mkdir -p $OUT
for s in 4 8 16 32 64 4 8 16 32 64; do
  timeout -k 10 180 python bench.py --seeds 256 --steps 6 --warmup 3 --no-cpu --streams $s > $OUT/s$s.log 2>&1 || exit $?
  grep '^{' $OUT/s$s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('streams', $s, round(d['value']/1e6,2), round(d['ms_per_step'],3), d['seeds_digest'][:16])"
done
echo done
