#!/bin/bash
# NN A/B runs (one MI355X); stops at the first failing step.
mkdir -p gpurun_out/m5
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >> gpurun_out/m5/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/m5/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> gpurun_out/m5/steps.log
  tail -c 300 "gpurun_out/m5/$name.log"; echo
  [ $rc -ne 0 ] && exit $rc
  return 0
}
run engine_tests 300 python -u -m pytest tests/test_engine_gpu.py tests/test_replay_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
B="python bench.py --steps 50 --warmup 5 --no-cpu"
run base 120 $B
export MPT_NN_BINNED=0; run nobin 120 $B; unset MPT_NN_BINNED
export MPT_NN1_FIRST_RING=1; run first1 120 $B; unset MPT_NN1_FIRST_RING
export MPT_NN_BINNED=0 MPT_NN1_GROUP=32 MPT_NN1_FIRST_RING=1; run nobin_g32f1 120 $B; unset MPT_NN_BINNED MPT_NN1_GROUP MPT_NN1_FIRST_RING
run base2 120 $B
run c5a 300 python bench.py --seeds 256 --steps 5 --warmup 3 --no-cpu
run c5b 300 python bench.py --seeds 256 --steps 5 --warmup 3 --no-cpu
echo all done
