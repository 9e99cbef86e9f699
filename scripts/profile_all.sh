#!/bin/bash
# Usage: TAG=r21 bash scripts/profile_all.sh [steps...]   (steps: c2 room snake c5_32 c5_256 prm
#        distance sq; default all -- split them over two calls to stay inside one call's limit)
# On the GPU box: rocprofv3 kernel trace + FETCH_SIZE + WRITE_SIZE passes (scripts/profile.sh)
# over every workload the bench line reports, summarised into gpurun_out/profiles_$TAG/<sub>/
# (pmc_summary.json = HBM bytes per launch, kernel_stats.csv), plus the SQ counters of config
# 5's tree walk.  Copy the result into profiles/$TAG/ to make bench.py read it.
TAG=${TAG:?set TAG}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/profiles_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
prof() {  # name script args window...
  local name=$1 script=$2 args=$3; shift 3
  SCRIPT=$script BENCH_ARGS="$args" bash scripts/profile.sh ${TAG}_$name || return 1
  python scripts/pmc_summary.py $R/gpurun_out/prof_${TAG}_$name $OUT/$name "$@" > /dev/null || return 1
  echo "$name done"
}
STEPS=("$@"); [ ${#STEPS[@]} -eq 0 ] && STEPS=(c2 room snake c5_32 c5_256 prm distance sq)
want() { local x; for x in "${STEPS[@]}"; do [ "$x" = "$1" ] && return 0; done; return 1; }
if want c2; then prof c2 bench.py "--steps 5 --warmup 2 --no-cpu --no-variants" || exit 1; fi
if want room; then prof room bench.py "--workload blimp-room --steps 5 --warmup 2 --no-cpu --no-variants" || exit 1; fi
if want snake; then prof snake bench.py "--workload snake --steps 5 --warmup 2 --no-cpu --no-variants" || exit 1; fi
if want c5_32; then prof c5_32 bench.py "--seeds 32 --steps 25 --warmup 5 --no-cpu" last:k_sample_jobs || exit 1; fi
if want c5_256; then prof c5_256 bench.py "--seeds 256 --steps 25 --warmup 5 --no-cpu" last:k_sample_jobs || exit 1; fi
if want prm; then prof prm scripts/bench_prm.py "--reps 1 --no-cpu" last:k_sort_segments || exit 1; fi
if want distance; then prof distance scripts/bench_distance.py "--steps 3 --warmup 1 --no-cpu" || exit 1; fi
want sq || { echo profile_all done; exit 0; }
# SQ counters of the kernels the verdict asks about (one pass each, 8 SQ counters): wait / issue
# split (the guide: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES)
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"
sq() {  # name kernel mode units script args...
  local name=$1 kern=$2 mode=$3 units=$4 script=$5; shift 5
  timeout -s KILL 240 rocprofv3 --pmc $SQ --output-format csv -d $R/gpurun_out/prof_${TAG}_sq_$name -o run -- python3 $R/$script "$@" > $OUT/sq_$name.log 2>&1 || return 1
  python3 scripts/sq_summary.py $R/gpurun_out/prof_${TAG}_sq_$name/run_counter_collection.csv $OUT/sq_$name.json "$kern" $mode $units > /dev/null || return 1
  rm -f $R/gpurun_out/prof_${TAG}_sq_$name/run_counter_collection.csv
  echo "sq $name done"
}
sq ct_nn1_jobs k_ct_nn1_jobs last 1048576 bench.py --seeds 256 --steps 25 --warmup 5 --no-cpu || exit 1
sq grid_nn1 k_grid_nn1_runs_sorted all 65536 bench.py --steps 5 --warmup 2 --no-cpu --no-variants || exit 1
sq cands_room k_cands all "" bench.py --workload blimp-room --steps 5 --warmup 2 --no-cpu --no-variants || exit 1
sq distance k_distance all 65536 scripts/bench_distance.py --steps 3 --warmup 1 --no-cpu || exit 1
sq sweep_prm "k_sweep_prm<1024" all "" scripts/bench_prm.py --reps 1 --no-cpu || exit 1
echo profile_all done
