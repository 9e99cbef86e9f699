#!/bin/bash
# Joint NN launch (mpt_rrt_step_many): parity tests, then config 5 joint vs per-seed, then a kernel trace.
OUT=gpurun_out/ab5c; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_prm_connect_gpu.py tests/test_nn_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
B="python bench.py --seeds 256 --steps 8 --warmup 3 --no-cpu"
for j in joint; do
  X=""; [ $j = solo ] && X="--no-joint-nn"
  timeout -k 10 180 $B $X > $OUT/$j.log 2>&1 || exit $?
  grep '^{' $OUT/$j.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$j', round(d['value']/1e6,2), round(d['ms_per_step'],3), d['seeds_digest'][:16])"
done
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py --seeds 256 --steps 4 --warmup 2 --no-cpu > $OUT/kt.log 2>&1 || exit $?
echo done
