#!/bin/bash
# Plan folded into k_pt_bbox + config 5 roofline from the joint launch: parity, config 5, config 2.
OUT=gpurun_out/ab5d; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_prm_connect_gpu.py tests/test_nn_gpu.py tests/test_prm_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 180 python bench.py --seeds 256 --steps 8 --warmup 3 --no-cpu > $OUT/c5.log 2>&1 || exit $?
grep '^{' $OUT/c5.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('c5', round(d['value']/1e6,2), round(d['ms_per_step'],3), d['seeds_digest'][:16], r['kernel'], r['ms_per_launch'], r['achieved'], r['frac'])"
timeout -k 10 180 python bench.py --steps 30 --warmup 5 --no-cpu > $OUT/c2.log 2>&1 || exit $?
grep '^{' $OUT/c2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', round(d['value']/1e6,2), round(d['ms_per_step'],4))"
echo done
