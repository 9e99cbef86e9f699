#!/bin/bash
# One GPU session: parity tests, smoke, short bench.  Stops at the first step that ends
# in a fault/abort/timeout (exit status > 1); test failures (status 1) do not stop it.
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -4 "gpurun_out/$name.log"
  return $rc
}
run pytest_gpu 800 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider -ra --timeout 120 --timeout-method thread; rc=$?
[ $rc -gt 1 ] && exit $rc
run smoke 180 python -c "import __graft_entry__ as g; g.smoke()"; rc=$?
[ $rc -gt 1 ] && exit $rc
run bench 400 python bench.py --steps 10 --warmup 3 --cpu-seconds 5 ${BENCH_EXTRA}; rc=$?
[ $rc -gt 1 ] && exit $rc
[ -n "$BENCH2" ] && { run bench2 400 python bench.py --steps 5 --warmup 2 --no-cpu $BENCH2; rc=$?; }
exit $rc
