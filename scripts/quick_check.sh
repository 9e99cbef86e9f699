#!/bin/bash
# Full GPU parity suite, then a kernel trace of the default bench (per-kernel times over the
# timed rounds) and bench lines for the workloads in $WORKLOADS.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/qc
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider -ra --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu > $OUT/kt.log 2>&1 || { tail $OUT/kt.log; exit 1; }
python scripts/trace_rounds.py $OUT/kt/run_kernel_trace.csv --warmup 3 --steps 20 --json $OUT/timed_rounds.json > $OUT/timed_rounds.txt 2>&1; cat $OUT/timed_rounds.txt
rm -f $OUT/kt/run_kernel_trace.csv
for w in ${WORKLOADS:-blimp}; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu > $OUT/bench_$w.log 2>&1 || { tail $OUT/bench_$w.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(sys.argv[2], round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],4), 'ms', d['kernel_ms_per_round'])" $OUT/bench_$w.log $w
done
echo done
