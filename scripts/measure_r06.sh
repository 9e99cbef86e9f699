#!/bin/bash
# Round-1 (third session) measurements on one MI355X: config 2 / 3 / 5 bench lines, then the
# rocprofv3 passes of config 2 (kernel trace + stats, FETCH_SIZE, WRITE_SIZE).  Every GPU step
# has its own time limit; the script stops at the first failure.
OUT=gpurun_out/m13
mkdir -p $OUT
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
run c5 300 python bench.py --seeds 256 --steps 5 --warmup 3 --no-cpu
run c2 300 python bench.py --steps 30 --warmup 5 --cpu-seconds 15
run c3 300 python bench.py --workload snake --steps 20 --warmup 3 --cpu-seconds 10
BENCH_ARGS="--steps 20 --warmup 3 --no-cpu" bash scripts/profile.sh r06 || exit $?
python scripts/pmc_summary.py gpurun_out/prof_r06 $OUT/r06 > $OUT/pmc.log 2>&1
python scripts/trace_rounds.py gpurun_out/prof_r06/kt/run_kernel_trace.csv --warmup 3 --steps 20 --json $OUT/r06/timed_rounds.json > $OUT/rounds.txt 2>&1
echo all done
