#!/bin/bash
# Usage: TAG=r24 bash scripts/verify_distance.sh  (on the GPU box)
# After a k_distance change: the GPU suite, smoke() and the bench line (scripts/verify.sh),
# then the distance leg's profiles (kernel trace + FETCH_SIZE + WRITE_SIZE passes) and its SQ
# pass, into gpurun_out/profiles_$TAG/.
TAG=${TAG:?set TAG}
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash scripts/verify.sh || exit 1
bash scripts/profile_all.sh distance || exit 1
OUT=$R/gpurun_out/profiles_$TAG
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"
timeout -s KILL 240 rocprofv3 --pmc $SQ --output-format csv -d $R/gpurun_out/prof_${TAG}_sq_distance -o run -- python3 $R/scripts/bench_distance.py --steps 3 --warmup 1 --no-cpu > $OUT/sq_distance.log 2>&1 || exit 1
python3 scripts/sq_summary.py $R/gpurun_out/prof_${TAG}_sq_distance/run_counter_collection.csv $OUT/sq_distance.json k_distance all 65536 > /dev/null || exit 1
rm -f $R/gpurun_out/prof_${TAG}_sq_distance/run_counter_collection.csv
echo verify_distance done
