#!/bin/bash
# Usage: TAG=r20 bash scripts/verify.sh [pytest selection args...]
# On the GPU box: the GPU test suite, smoke() and the default bench line, each under its own
# time limit; stops at the first failure.  Logs and the bench line under gpurun_out/verify_$TAG/.
TAG=${TAG:?set TAG}
OUT=gpurun_out/verify_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> $OUT/steps.log
  tail -c 600 "$OUT/$name.log"; echo
  [ $rc -ne 0 ] && exit $rc
  return 0
}
SEL=("$@")
[ ${#SEL[@]} -eq 0 ] && SEL=(tests)
step pytest 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "${SEL[@]}"
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
if [ -z "$NO_BENCH" ]; then
  step bench 900 python bench.py
  grep '^{' $OUT/bench.log > $OUT/bench.json
fi
echo verify done
