#!/bin/bash
# End-of-session check on one MI355X: every GPU test, smoke, config 2 and config 5 bench lines
# (5 and 30 rounds), and the kernel trace of the 6-round config 5 command.
OUT=gpurun_out/m17
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> $OUT/steps.log
  tail -c 200 "$OUT/$name.log"; echo
  [ $rc -ne 0 ] && exit $rc
  return 0
}
run tests 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
run smoke 180 python -c "import __graft_entry__ as g; g.smoke()"
run c2 300 python bench.py --steps 30 --warmup 5 --cpu-seconds 15
run c5 300 python bench.py --seeds 256 --steps 6 --warmup 3 --no-cpu
run c5_30 300 python bench.py --seeds 256 --steps 30 --warmup 3 --no-cpu
run kt 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py --seeds 256 --steps 6 --warmup 3 --no-cpu
rm -f $OUT/kt/run_kernel_trace.csv
for c in c2 c5 c5_30; do grep '^{' $OUT/$c.log > $OUT/bench_$c.json; done
echo all done
