#!/bin/bash
# Config 3 (snake) NN structure comparison + config 2 default check (one MI355X).
mkdir -p gpurun_out/m6
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >> gpurun_out/m6/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/m6/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> gpurun_out/m6/steps.log
  tail -c 300 "gpurun_out/m6/$name.log"; echo
  [ $rc -ne 0 ] && exit $rc
  return 0
}
run nn_tests 300 python -u -m pytest tests/test_nn_gpu.py tests/test_engine_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run c2 120 python bench.py --steps 50 --warmup 5 --no-cpu
S="python bench.py --workload snake --steps 10 --warmup 3 --no-cpu"
run snake_auto 200 $S
run snake_tree 200 $S --nn tree
run snake_brute 200 $S --nn brute
run snake_ppc8 200 $S --nn grid --ppc 8
run snake_ppc05 200 $S --nn grid --ppc 0.5
echo all done
