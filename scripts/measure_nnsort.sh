#!/bin/bash
# Sorted-query grid 1-NN (QueryOrder): engine + NN parity tests, A/B against the unsorted
# launch, then SQ counter passes of the NN kernel (scripts/sq_profile.sh).  Stops at the
# first failure.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TESTS:-tests/test_engine_gpu.py tests/test_nn_gpu.py tests/test_scale_gpu.py}
timeout -k 10 400 python -u -m pytest $T -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/nnsort_tests.log 2>&1 || { tail -20 gpurun_out/nnsort_tests.log; exit 1; }
tail -2 gpurun_out/nnsort_tests.log
bash scripts/ab.sh nnsort_c2 "sort:" "nosort:MPT_NN_SORT=0" || exit 1
BENCH_ARGS="--workload snake --steps 10 --warmup 3 --no-cpu" bash scripts/ab.sh nnsort_snake "sort:" "nosort:MPT_NN_SORT=0" || exit 1
if [ -n "$SQ" ]; then
  KERNEL='k_grid_nn1_runs' bash scripts/sq_profile.sh sqnn > gpurun_out/sqnn.log 2>&1 || { tail gpurun_out/sqnn.log; exit 1; }
  python scripts/sq_summary.py gpurun_out/prof_sqnn gpurun_out/sqnn.json > gpurun_out/sqnn_summary.txt 2>&1; cat gpurun_out/sqnn_summary.txt
  find gpurun_out/prof_sqnn -name "*.csv" -size +5M -delete
fi
echo done
