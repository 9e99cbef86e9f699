#!/bin/bash
# Usage: TAG=r21 bash scripts/profile_all.sh
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
  rm -rf $R/gpurun_out/prof_${TAG}_$name/kt/*_kernel_trace.csv
  echo "$name done"
}
prof c2 bench.py "--steps 5 --warmup 2 --no-cpu --no-variants" || exit 1
prof room bench.py "--workload blimp-room --steps 5 --warmup 2 --no-cpu --no-variants" || exit 1
prof snake bench.py "--workload snake --steps 5 --warmup 2 --no-cpu --no-variants" || exit 1
prof c5_32 bench.py "--seeds 32 --steps 25 --warmup 5 --no-cpu" last:k_sample_jobs || exit 1
prof c5_256 bench.py "--seeds 256 --steps 25 --warmup 5 --no-cpu" last:k_sample_jobs || exit 1
prof prm scripts/bench_prm.py "--reps 1 --no-cpu" last:k_sort_segments || exit 1
prof distance scripts/bench_distance.py "--steps 3 --warmup 1 --no-cpu" || exit 1
# the tree walk's instruction and wait counters (one pass: 5 SQ counters)
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv \
  -d $R/gpurun_out/prof_${TAG}_sq -o run -- python3 bench.py --seeds 256 --steps 25 --warmup 5 --no-cpu > $OUT/sq.log 2>&1 || exit 1
python - $R/gpurun_out/prof_${TAG}_sq/run_counter_collection.csv $OUT/sq_ct_nn1_jobs.json <<'PY'
import csv, json, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_ct_nn1_jobs" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Dispatch_Id"]))
last = max(int(r["Dispatch_Id"]) for r in rows)
agg = collections.defaultdict(float)
for r in rows:
    if int(r["Dispatch_Id"]) == last:
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
out = {"kernel": "k_ct_nn1_jobs<7, 64, 8> (the last joint round of bench.py --seeds 256 --steps 25 --warmup 5)",
       "queries": 256 * 4096, **agg}
q = out["queries"]
if agg.get("SQ_INSTS_VALU"):
    # SQ_INSTS_VALU counts wave instructions; one query is one wave
    out["valu_instructions_per_query"] = agg["SQ_INSTS_VALU"] / q
if agg.get("SQ_WAVE_CYCLES"):
    out["wait_any_over_wave_cycles"] = agg.get("SQ_WAIT_ANY", 0) / agg["SQ_WAVE_CYCLES"]
json.dump(out, open(sys.argv[2], "w"), indent=1)
print(json.dumps(out))
PY
rm -f $R/gpurun_out/prof_${TAG}_sq/run_counter_collection.csv.bak
echo profile_all done
