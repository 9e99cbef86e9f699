#!/bin/bash
# Usage: TAG=r23 bash scripts/nn_traffic.sh [seeds]
# On the GPU box: scripts/nn_traffic.py under a kernel trace and one PMC pass each for
# FETCH_SIZE and WRITE_SIZE, summarised by scripts/nn_traffic_summary.py into
# gpurun_out/nn_traffic_$TAG/summary.json (copy into profiles/ to keep it).
TAG=${TAG:?set TAG}
SEEDS=${1:-256}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/nn_traffic_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 $R/scripts/nn_traffic.py --seeds $SEEDS --out $OUT/replay_kt.json > $OUT/kt.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $R/scripts/nn_traffic.py --seeds $SEEDS --out $OUT/replay_fetch.json > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $R/scripts/nn_traffic.py --seeds $SEEDS --out $OUT/replay_write.json > $OUT/write.log 2>&1 || exit $?
python3 $R/scripts/nn_traffic_summary.py $OUT > $OUT/summary.log 2>&1 || exit $?
rm -f $OUT/kt/*_kernel_trace.csv.bak
echo nn_traffic done
