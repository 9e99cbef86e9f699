#!/bin/bash
# Fused spread feedback + NN-distance cell floor: engine tests, config 2, snake sweep of the
# floor factor.  Every GPU step has its own time limit; stops at the first failure.
mkdir -p gpurun_out/m9
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >> gpurun_out/m9/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/m9/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> gpurun_out/m9/steps.log
  tail -c 300 "gpurun_out/m9/$name.log"; echo
  [ $rc -ne 0 ] && exit $rc
  return 0
}
run engine_tests 300 python -u -m pytest tests/test_engine_gpu.py tests/test_nn_gpu.py tests/test_replay_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run c2 120 python bench.py --steps 30 --warmup 5 --no-cpu
run c5s 200 python bench.py --seeds 64 --steps 3 --warmup 2 --no-cpu
run c5 300 python bench.py --seeds 256 --steps 5 --warmup 3 --no-cpu
S="python bench.py --workload snake --steps 10 --warmup 3 --no-cpu"
for k in 0.25 0.4 0.6 0.9; do export MPT_NN_HMIN_K=$k; run snake_k$k 200 $S; done; unset MPT_NN_HMIN_K
run snake_tree 200 $S --nn tree
echo all done
