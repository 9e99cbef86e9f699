#!/bin/bash
# Usage: TAG=x bash scripts/r21.sh [pytest files...]
# On the GPU box: the given GPU tests, then config 5 at 32 / 256 seeds (25 + 5 rounds) and
# config 4 at --bounds rooms; lines under gpurun_out/$TAG/.  Stops at the first failure.
TAG=${TAG:?set TAG}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -z "$NO_C5" ]; then
for n in 32 256; do
  timeout -k 10 200 python bench.py --seeds $n --steps 25 --warmup 5 --no-cpu --detail $O/c5_${n}_detail.json > $O/c5_$n.json || exit 1
done
fi
[ -n "$NO_PRM" ] || timeout -k 10 300 python scripts/bench_prm.py --reps 3 --no-cpu > $O/prm.json || exit 1
if [ -n "$SCRATCH" ]; then
  for w in none stream group; do
    for n in 32 256; do timeout -k 10 200 python scripts/scratch_rounds.py --seeds $n --warm $w > $O/scratch_${n}_$w.json || exit 1; cat $O/scratch_${n}_$w.json; done
  done
fi
if [ -n "$PRMKT" ]; then  # config 4's kernels
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prmkt -o kt -- python scripts/bench_prm.py --reps 1 --no-cpu > $O/prmkt.log 2>&1 || exit 1
  head -12 $O/prmkt/kt_kernel_stats.csv | cut -d, -f1-4
  rm -f $O/prmkt/kt_kernel_trace.csv
fi
if [ -n "$HIPT" ]; then  # HIP API time of a run from the start states (first-round costs)
  timeout -k 10 200 rocprofv3 --hip-trace --stats --output-format csv -d $O/hipt -o ht -- python scripts/scratch_rounds.py --seeds 32 --rounds 3 > $O/hipt.log 2>&1 || exit 1
fi
if [ -n "$KT" ]; then  # per-round kernel sums over rounds 10..19 of a kernel trace (scripts/kt_last.py)
  for n in 32 256; do
    timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/c$n -o kt -- python bench.py --seeds $n --steps 25 --warmup 5 --no-cpu --detail $O/kt_detail.json > $O/kt$n.log 2>&1 || exit 1
    python scripts/kt_last.py $O/c$n/kt_kernel_trace.csv --rounds k_sample_jobs 10 20 > $O/rounds_$n.txt || exit 1
    rm -f $O/c$n/kt_kernel_trace.csv
  done
fi
python - $O <<'PY'
import json, sys
o = sys.argv[1]
for n in (32, 256):
    try:
        d = json.load(open(f"{o}/c5_{n}_detail.json"))
    except OSError:
        continue
    st = {k: round(v.get("ms_event_free", v["ms"]), 3) for k, v in d["roofline"]["stages"].items()}
    print(n, round(d["value"] / 1e6, 1), "M/s", round(d["ms_per_step"], 3), "ms", d["seeds_digest"][:8],
          "scratch", round(d["from_scratch"]["valid_per_s"] / 1e6, 1), st)
try:
    p = json.loads(open(f"{o}/prm.json").read().strip().splitlines()[-1])
    print("prm", round(p["value"] / 1e6, 2), "M milestones/s", p["device_ms"], p["config"]["free_fraction"],
          p["roofline"].get("work"))
except Exception as e:
    print("prm", e)
PY
