#!/bin/bash
# Grid NN: XCD-slab variant vs default (parity tests under the knob, then config 2 / 3 A/B).
OUT=gpurun_out/abx; mkdir -p $OUT
export MPT_NN1_XCD=1
timeout -k 10 300 python -u -m pytest tests/test_nn_gpu.py tests/test_engine_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests_xcd.log 2>&1 || exit $?
B="python bench.py --steps 30 --warmup 5 --no-cpu"
timeout -k 10 120 $B > $OUT/c2_xcd.log 2>&1 || exit $?
timeout -k 10 200 $B --workload snake > $OUT/c3_xcd.log 2>&1 || exit $?
unset MPT_NN1_XCD
timeout -k 10 120 $B > $OUT/c2_base.log 2>&1 || exit $?
timeout -k 10 200 $B --workload snake > $OUT/c3_base.log 2>&1 || exit $?
echo done
