#!/bin/bash
# Round-1 (fourth session) measurements on one MI355X: GPU tests + smoke, rocprofv3 passes of
# config 2 and config 5 (kernel trace + stats, FETCH_SIZE, WRITE_SIZE), the PMC summary, then
# the config 2 / 3 / 5 bench lines (which read that summary for their `traffic` fields).
# Every GPU step has its own time limit; the script stops at the first failure.
OUT=gpurun_out/m14
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
run smoke 180 python -c "import __graft_entry__ as g; g.smoke()"
BENCH_ARGS="--steps 20 --warmup 3 --no-cpu" bash scripts/profile.sh r07 || exit $?
BENCH_ARGS="--seeds 256 --steps 6 --warmup 3 --no-cpu" bash scripts/profile.sh r07c5 || exit $?
python scripts/pmc_summary.py gpurun_out/prof_r07 $OUT/r07 > $OUT/pmc.log 2>&1 || exit 1
python scripts/pmc_summary.py gpurun_out/prof_r07c5 $OUT/r07/c5 > $OUT/pmc_c5.log 2>&1 || exit 1
mkdir -p profiles/r07 && OUT=$OUT python - <<'PY' || exit 1
import json, os
o = os.environ["OUT"]
a = json.load(open(o + "/r07/pmc_summary.json"))
b = json.load(open(o + "/r07/c5/pmc_summary.json"))
for k, v in b.items():
    a.setdefault(k, v)  # config 5's own kernels (k_tree_nn1_jobs, the tree build)
json.dump(a, open(o + "/r07/pmc_summary.json", "w"), indent=1)
json.dump(a, open("profiles/r07/pmc_summary.json", "w"), indent=1)  # what bench.py reads
PY
python scripts/trace_rounds.py gpurun_out/prof_r07/kt/run_kernel_trace.csv --warmup 3 --steps 20 --json $OUT/r07/timed_rounds.json > $OUT/rounds.txt 2>&1
run c2 300 python bench.py --steps 30 --warmup 5 --cpu-seconds 15
run c3 300 python bench.py --workload snake --steps 20 --warmup 3 --cpu-seconds 10
run c5 300 python bench.py --seeds 256 --steps 30 --warmup 3 --no-cpu
for c in c2 c3 c5; do grep '^{' $OUT/$c.log > $OUT/r07/bench_$c.json; done
python scripts/trace_rounds.py gpurun_out/prof_r07c5/kt/run_kernel_trace.csv > $OUT/rounds_c5.txt 2>&1
# the raw traces and counter rows exceed what gpurun copies back; the summaries stay
find gpurun_out/prof_r07 gpurun_out/prof_r07c5 -name "run_kernel_trace.csv" -delete
find gpurun_out/prof_r07 gpurun_out/prof_r07c5 -name "run_counter_collection.csv" -delete
du -sh gpurun_out
echo all done
