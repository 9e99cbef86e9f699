#!/bin/bash
# k_cands waves per CU (config 2 and 3) + the blimp steer reuse check (engine tests).
OUT=gpurun_out/abc; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_replay_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit $?
B="python bench.py --steps 40 --warmup 5 --no-cpu"
for w in 16 32 64; do
  timeout -k 10 120 env MPT_CANDS_WAVES_PER_CU=$w $B > $OUT/c2_w$w.log 2>&1 || exit $?
  timeout -k 10 200 env MPT_CANDS_WAVES_PER_CU=$w $B --workload snake > $OUT/c3_w$w.log 2>&1 || exit $?
done
echo done
