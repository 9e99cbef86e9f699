#!/bin/bash
# Usage: TAG=r10 bash scripts/measure_round.sh
# Round-2 measurements (second session) on one MI355X: rocprofv3 passes (kernel trace + stats, FETCH_SIZE,
# WRITE_SIZE) of config 2, its collision-heavy variant and config 5, their PMC summaries (per
# workload: the same kernel names carry different traffic in each), then the bench lines,
# each reading its own workload's summary.  Every GPU step has its own time limit; the script
# stops at the first failure.
TAG=${TAG:?set TAG}
OUT=gpurun_out/m_$TAG
P=$OUT/$TAG  # copied to profiles/$TAG afterwards
mkdir -p $OUT $P
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> $OUT/steps.log
  tail -c 400 "$OUT/$name.log"; echo
  [ $rc -ne 0 ] && exit $rc
  return 0
}
BENCH_ARGS="--steps 20 --warmup 3 --no-cpu" bash scripts/profile.sh $TAG || exit $?
BENCH_ARGS="--workload blimp-room --steps 20 --warmup 3 --no-cpu" bash scripts/profile.sh ${TAG}room || exit $?
BENCH_ARGS="--seeds 256 --steps 6 --warmup 3 --no-cpu" bash scripts/profile.sh ${TAG}c5 || exit $?
BENCH_ARGS="--workload snake --steps 10 --warmup 3 --no-cpu" bash scripts/profile.sh ${TAG}snake || exit $?
python scripts/pmc_summary.py gpurun_out/prof_$TAG $P > $OUT/pmc.log 2>&1 || exit 1
python scripts/pmc_summary.py gpurun_out/prof_${TAG}room $P/room > $OUT/pmc_room.log 2>&1 || exit 1
python scripts/pmc_summary.py gpurun_out/prof_${TAG}c5 $P/c5 > $OUT/pmc_c5.log 2>&1 || exit 1
python scripts/pmc_summary.py gpurun_out/prof_${TAG}snake $P/snake > $OUT/pmc_snake.log 2>&1 || exit 1
python scripts/trace_rounds.py gpurun_out/prof_$TAG/kt/run_kernel_trace.csv --warmup 3 --steps 20 --json $P/timed_rounds.json > $P/timed_rounds.txt 2>&1
python scripts/trace_rounds.py gpurun_out/prof_${TAG}room/kt/run_kernel_trace.csv --warmup 3 --steps 20 --json $P/room/timed_rounds.json > $P/room/timed_rounds.txt 2>&1
run c2 300 python bench.py --steps 30 --warmup 5 --cpu-seconds 15 --traffic $P/pmc_summary.json
run room 300 python bench.py --workload blimp-room --steps 30 --warmup 5 --cpu-seconds 15 --traffic $P/room/pmc_summary.json
run c5 300 python bench.py --seeds 256 --steps 30 --warmup 3 --no-cpu --traffic $P/c5/pmc_summary.json
run c5_32 300 python bench.py --seeds 32 --steps 30 --warmup 3 --no-cpu --traffic $P/c5/pmc_summary.json
run snake 300 python bench.py --workload snake --steps 20 --warmup 3 --cpu-seconds 15 --traffic $P/snake/pmc_summary.json
for c in c2 room c5 c5_32 snake; do grep '^{' $OUT/$c.log > $P/bench_$c.json; done
# the raw traces and counter rows exceed what gpurun copies back; the summaries stay
find gpurun_out/prof_$TAG gpurun_out/prof_${TAG}room gpurun_out/prof_${TAG}c5 gpurun_out/prof_${TAG}snake -name "run_kernel_trace.csv" -delete
find gpurun_out/prof_$TAG gpurun_out/prof_${TAG}room gpurun_out/prof_${TAG}c5 gpurun_out/prof_${TAG}snake -name "run_counter_collection.csv" -delete
du -sh gpurun_out
echo all done
