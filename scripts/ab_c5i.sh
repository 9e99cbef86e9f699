#!/bin/bash
# Joint tree build (one launch per stage + a segmented sort for all seeds): parity, then config 5.
OUT=gpurun_out/ab5i; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_prm_connect_gpu.py tests/test_nn_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2; do
  timeout -k 10 180 python bench.py --seeds 256 --steps 6 --warmup 3 --no-cpu > $OUT/c5_$i.log 2>&1 || { tail -20 $OUT/c5_$i.log; exit 1; }
  grep '^{' $OUT/c5_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c5', round(d['value']/1e6,2), round(d['ms_per_step'],3), d['seeds_digest'][:16], r['ms_per_launch'])"
done
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py --seeds 256 --steps 6 --warmup 3 --no-cpu > $OUT/kt.log 2>&1 || exit $?
rm -f $OUT/kt/run_kernel_trace.csv
echo done
