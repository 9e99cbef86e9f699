#!/bin/bash
# rocprofv3 passes over the default bench workload: kernel trace + stats, then one PMC
# pass per TCC counter (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950).
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
ARGS=${BENCH_ARGS:---steps 5 --warmup 2 --no-cpu}
SCRIPT=${SCRIPT:-bench.py}  # e.g. SCRIPT=scripts/bench_prm.py
mkdir -p $R/gpurun_out
set -o pipefail
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG/kt -o run -- python3 $R/$SCRIPT $ARGS > $R/gpurun_out/prof_${TAG}_kt.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof_$TAG/fetch -o run -- python3 $R/$SCRIPT $ARGS > $R/gpurun_out/prof_${TAG}_fetch.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof_$TAG/write -o run -- python3 $R/$SCRIPT $ARGS > $R/gpurun_out/prof_${TAG}_write.log 2>&1 || exit $?
echo profile done
