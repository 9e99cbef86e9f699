#!/bin/bash
# Usage: TAG=r23 bash scripts/final_profiles.sh  (on the GPU box)
# The head's config-5 profiles (kernel trace + FETCH + WRITE), the SQ passes of the tree walk
# and the PRM sweep, and the NN traffic replay at 256 seeds.
TAG=${TAG:?set TAG}
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash scripts/profile_all.sh c5_32 c5_256 || exit 1
OUT=$R/gpurun_out/profiles_$TAG
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"
for spec in "ct_nn1_jobs|k_ct_nn1_jobs|last|1048576|bench.py --seeds 256 --steps 25 --warmup 5 --no-cpu" \
            "sweep_prm|k_sweep_prm<1024|all||scripts/bench_prm.py --reps 1 --no-cpu"; do
  IFS='|' read -r name kern mode units cmd <<< "$spec"
  timeout -s KILL 240 rocprofv3 --pmc $SQ --output-format csv -d $R/gpurun_out/prof_${TAG}_sq_$name -o run -- python3 $R/$cmd > $OUT/sq_$name.log 2>&1 || exit 1
  python3 scripts/sq_summary.py $R/gpurun_out/prof_${TAG}_sq_$name/run_counter_collection.csv $OUT/sq_$name.json "$kern" $mode $units > /dev/null || exit 1
  rm -f $R/gpurun_out/prof_${TAG}_sq_$name/run_counter_collection.csv
  echo "sq $name done"
done
TAG=${TAG}f bash scripts/nn_traffic.sh 256 || exit 1
echo final_profiles done
