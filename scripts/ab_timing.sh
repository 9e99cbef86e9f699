#!/bin/bash
# Cost of recording the per-stage hipEvents inside the timed rounds (config 2, one MI355X).
OUT=gpurun_out/abt; mkdir -p $OUT
for e in 1 4 0 1; do
  timeout -k 10 120 python bench.py --steps 60 --warmup 5 --no-cpu --stage-every $e > $OUT/every$e.log 2>&1 || exit $?
  grep '^{' $OUT/every$e.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('every', $e, round(d['value']/1e6,2), round(d['ms_per_step'],4))"
done
