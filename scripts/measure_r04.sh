#!/bin/bash
# Round-1 (second session) measurements on one MI355X: default bench (config 2), config 3
# (snake), config 5 (256 seeds), an NN knob sweep, then the rocprofv3 passes of config 2.
# Every GPU step has its own time limit; the script stops at the first fault/abort/timeout.
mkdir -p gpurun_out/m4
cd "${GRAFT_REPO_ROOT:-.}"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >> gpurun_out/m4/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/m4/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> gpurun_out/m4/steps.log
  tail -c 600 "gpurun_out/m4/$name.log"; echo
  [ $rc -ne 0 ] && exit $rc
  return 0
}
run c2 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 15
run c3 300 python bench.py --workload snake --steps 20 --warmup 3 --cpu-seconds 10
run c5 300 python bench.py --seeds 256 --steps 5 --warmup 3 --no-cpu
for g in 8 32; do export MPT_NN1_GROUP=$g; run grp$g 120 python bench.py --steps 20 --warmup 3 --no-cpu; done; unset MPT_NN1_GROUP
export MPT_NN1_FIRST_RING=1; run first1 120 python bench.py --steps 20 --warmup 3 --no-cpu; unset MPT_NN1_FIRST_RING
for p in 1 4; do run ppc$p 120 python bench.py --steps 20 --warmup 3 --no-cpu --ppc $p; done
TAG=r04 BENCH_ARGS="--steps 20 --warmup 3 --no-cpu" bash scripts/profile.sh r04 || exit $?
python scripts/pmc_summary.py gpurun_out/prof_r04 gpurun_out/m4/r04 > gpurun_out/m4/pmc.log 2>&1
echo all done
