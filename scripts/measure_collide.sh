#!/bin/bash
# Collision-path changes: collide + engine parity tests, then A/B bench lines ("NAME:ENV=VAL")
# on config 2 and the collision-heavy room.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
T=${TESTS:-tests/test_collide_gpu.py tests/test_engine_gpu.py}
timeout -k 10 500 python -u -m pytest $T -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/collide_tests.log 2>&1 || { tail -20 gpurun_out/collide_tests.log; exit 1; }
tail -1 gpurun_out/collide_tests.log
bash scripts/ab.sh col_c2 "$@" || exit 1
BENCH_ARGS="--workload blimp-room --steps 20 --warmup 3 --no-cpu" bash scripts/ab.sh col_room "$@" || exit 1
