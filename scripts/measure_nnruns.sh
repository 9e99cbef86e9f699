#!/bin/bash
# Grid NN: cell-run kernel vs the cell-per-lane walk, group/points-per-step variants (one MI355X).
mkdir -p gpurun_out/m10
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >> gpurun_out/m10/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/m10/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> gpurun_out/m10/steps.log
  tail -c 300 "gpurun_out/m10/$name.log"; echo
  [ $rc -ne 0 ] && exit $rc
  return 0
}
run nn_tests 300 python -u -m pytest tests/test_nn_gpu.py tests/test_engine_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
B="python bench.py --steps 30 --warmup 5 --no-cpu"
S="python bench.py --workload snake --steps 10 --warmup 3 --no-cpu"
run c2_runs32x2 120 $B
export MPT_NN1_PTS=1; run c2_runs32x1 120 $B; unset MPT_NN1_PTS
export MPT_NN1_GROUP=16; run c2_runs16x2 120 $B
export MPT_NN1_PTS=1; run c2_runs16x1 120 $B; unset MPT_NN1_PTS MPT_NN1_GROUP
export MPT_NN1_KERNEL=cells; run c2_cells 120 $B; run snake_cells 200 $S; unset MPT_NN1_KERNEL
run snake_runs32x2 200 $S
export MPT_NN1_GROUP=16; run snake_runs16x2 200 $S; unset MPT_NN1_GROUP
echo all done
