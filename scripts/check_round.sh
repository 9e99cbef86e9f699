#!/bin/bash
# Parity tests of the engine / collision / NN paths, config 2 bench, kernel trace of config 2
# (one MI355X).  OUT=gpurun_out/<dir>; stops at the first failing step.
OUT=${OUT:-gpurun_out/chk}
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> $OUT/steps.log
  tail -c 300 "$OUT/$name.log"; echo
  [ $rc -ne 0 ] && exit $rc
  return 0
}
run tests 600 python -u -m pytest ${TESTS:-tests/test_engine_gpu.py tests/test_collide_gpu.py tests/test_nn_gpu.py tests/test_replay_gpu.py} -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run c2 120 python bench.py --steps 30 --warmup 5 --no-cpu
[ -n "$EXTRA" ] && { run extra 300 $EXTRA; }
run kt 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu
python scripts/trace_rounds.py $OUT/kt/run_kernel_trace.csv > $OUT/rounds.txt 2>&1
echo all done
