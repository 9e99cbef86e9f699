#!/bin/bash
# Round-3 measurements on one MI355X.  PART=a: rocprofv3 passes (kernel trace + stats, FETCH_SIZE,
# WRITE_SIZE) of config 2, blimp-room, snake and config 5 at 32 and 256 seeds -- each at the
# same rounds as its bench line -- and their PMC summaries (copy them to profiles/$TAG before
# PART=b: every gpurun call starts on a fresh box).  PART=b: config 4 (scripts/bench_prm.py)
# passes, then the bench lines of configs 2, 3, 4 and blimp-room, each reading its own
# workload's summary.  PART=c: config 5's passes (joint rounds only) and bench lines.  Every GPU step has
# its own time limit; the script stops at the first failure.
#   TAG=r16 PART=a bash scripts/measure_r3.sh && TAG=r16 PART=b bash scripts/measure_r3.sh
# (C5=1 with PART=b: also config 5's bench lines, from part a's committed c5 summaries)
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
  tail -c 300 "$OUT/$name.log"; echo
  [ $rc -ne 0 ] && exit $rc
  return 0
}
summ() {  # tag dst [window-start window-end]
  python scripts/pmc_summary.py gpurun_out/prof_$1 $2 "${@:3}" > $OUT/pmc_$1.log 2>&1 || exit 1
}
if [ "${PART:-a}" = a ]; then
  BENCH_ARGS="--steps 30 --warmup 5 --no-cpu --no-variants" bash scripts/profile.sh ${TAG} || exit $?
  BENCH_ARGS="--workload blimp-room --steps 20 --warmup 3 --no-cpu --no-variants" bash scripts/profile.sh ${TAG}room || exit $?
  BENCH_ARGS="--workload snake --steps 10 --warmup 3 --no-cpu --no-variants" bash scripts/profile.sh ${TAG}snake || exit $?
  BENCH_ARGS="--seeds 32 --steps 30 --warmup 5 --no-cpu" bash scripts/profile.sh ${TAG}c5_32 || exit $?
  BENCH_ARGS="--seeds 256 --steps 30 --warmup 5 --no-cpu" bash scripts/profile.sh ${TAG}c5_256 || exit $?
  summ $TAG $P; summ ${TAG}room $P/room; summ ${TAG}snake $P/snake; summ ${TAG}c5_32 $P/c5_32 last:k_sample_jobs; summ ${TAG}c5_256 $P/c5_256 last:k_sample_jobs
  python scripts/trace_rounds.py gpurun_out/prof_$TAG/kt/run_kernel_trace.csv --warmup 5 --steps 30 --json $P/timed_rounds.json > $P/timed_rounds.txt 2>&1
  python scripts/trace_rounds.py gpurun_out/prof_${TAG}room/kt/run_kernel_trace.csv --warmup 3 --steps 20 --json $P/room/timed_rounds.json > $P/room/timed_rounds.txt 2>&1
  # the raw traces and counter rows exceed what gpurun copies back; the summaries stay
  find gpurun_out/prof_${TAG}* -name "run_kernel_trace.csv" -delete
  find gpurun_out/prof_${TAG}* -name "run_counter_collection.csv" -delete
  echo part a done
elif [ "${PART}" = c ]; then
  BENCH_ARGS="--seeds 32 --steps 30 --warmup 5 --no-cpu" bash scripts/profile.sh ${TAG}c5_32 || exit $?
  BENCH_ARGS="--seeds 256 --steps 30 --warmup 5 --no-cpu" bash scripts/profile.sh ${TAG}c5_256 || exit $?
  summ ${TAG}c5_32 $P/c5_32 last:k_sample_jobs; summ ${TAG}c5_256 $P/c5_256 last:k_sample_jobs
  find gpurun_out/prof_${TAG}c5* -name "run_kernel_trace.csv" -delete
  find gpurun_out/prof_${TAG}c5* -name "run_counter_collection.csv" -delete
  run c5_32 300 python bench.py --seeds 32 --traffic $P/c5_32/pmc_summary.json
  run c5_256 300 python bench.py --seeds 256 --traffic $P/c5_256/pmc_summary.json
  for c in c5_32 c5_256; do grep '^{' $OUT/$c.log > $P/bench_$c.json; done
  echo part c done
else
  SCRIPT=scripts/bench_prm.py BENCH_ARGS="--no-cpu --reps 2" bash scripts/profile.sh ${TAG}prm || exit $?
  summ ${TAG}prm $P/prm
  find gpurun_out/prof_${TAG}prm -name "run_kernel_trace.csv" -delete
  find gpurun_out/prof_${TAG}prm -name "run_counter_collection.csv" -delete
  # part a's summaries were made on another box: read the committed copies (profiles/$TAG)
  R=profiles/$TAG
  run c2 600 python bench.py --traffic $R/pmc_summary.json
  run room 300 python bench.py --workload blimp-room --steps 30 --warmup 5 --cpu-seconds 15 --no-variants --traffic $R/room/pmc_summary.json
  run snake 300 python bench.py --workload snake --steps 20 --warmup 3 --cpu-seconds 15 --no-variants --traffic $R/snake/pmc_summary.json
  run prm 300 python scripts/bench_prm.py --traffic $P/prm/pmc_summary.json
  for c in c2 room snake prm; do grep '^{' $OUT/$c.log > $P/bench_$c.json; done
  # config 5's lines from part a's summaries (PART=c re-profiles them instead)
  if [ -n "$C5" ]; then
    run c5_32 300 python bench.py --seeds 32 --traffic $R/c5_32/pmc_summary.json
    run c5_256 300 python bench.py --seeds 256 --traffic $R/c5_256/pmc_summary.json
    for c in c5_32 c5_256; do grep '^{' $OUT/$c.log > $P/bench_$c.json; done
  fi
  echo part b done
fi
du -sh gpurun_out
