#!/bin/bash
# Round-1 (third session): rocprofv3 passes of config 2 at HEAD, then config 3 (snake) NN
# structure comparison.  Every GPU step has its own time limit; stops at the first failure.
mkdir -p gpurun_out/m7
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >> gpurun_out/m7/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/m7/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> gpurun_out/m7/steps.log
  tail -c 300 "gpurun_out/m7/$name.log"; echo
  [ $rc -ne 0 ] && exit $rc
  return 0
}
BENCH_ARGS="--steps 20 --warmup 3 --no-cpu" bash scripts/profile.sh r05 || exit $?
python scripts/pmc_summary.py gpurun_out/prof_r05 gpurun_out/m7/r05 > gpurun_out/m7/pmc.log 2>&1
S="python bench.py --workload snake --steps 10 --warmup 3 --no-cpu"
run snake_auto 200 $S
run snake_tree 200 $S --nn tree
run snake_ppc8 200 $S --nn grid --ppc 8
run snake_ppc32 200 $S --nn grid --ppc 32
echo all done
