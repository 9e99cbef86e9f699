#!/bin/bash
# Usage: TAG=x bash scripts/ab_c5.sh [pytest selection...]
# On the GPU box: the given GPU tests, then config 5 at 32 and 256 seeds (25 + 5 rounds): bench
# lines and per-round kernel sums (rounds 10..19 of a kernel trace) under gpurun_out/ab_$TAG/.
TAG=${TAG:?set TAG}
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "$@" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
  tail -n 1 $OUT/pytest.log
fi
for n in 32 256; do
  timeout -k 10 200 python bench.py --seeds $n --steps 25 --warmup 5 --no-cpu > $OUT/c5_$n.json || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/c$n -o kt -- python bench.py --seeds $n --steps 25 --warmup 5 --no-cpu > $OUT/kt$n.log 2>&1 || exit 1
  python scripts/kt_last.py $OUT/c$n/kt_kernel_trace.csv --rounds k_sample_jobs 10 20 > $OUT/rounds_$n.txt || exit 1
  rm -f $OUT/c$n/kt_kernel_trace.csv
done
python - $OUT <<'PY'
import json, sys
out = sys.argv[1]
for n in (32, 256):
    d = json.loads(open(f"{out}/c5_{n}.json").read().strip().splitlines()[-1])
    top = open(f"{out}/rounds_{n}.txt").read().splitlines()[:4]
    print(n, round(d["value"] / 1e6, 1), "M/s", round(d["ms_per_step"], 3), "ms", d.get("seeds_digest", "")[:8])
    print("  " + "\n  ".join(top))
PY
