#!/bin/bash
# NN variants on the bench workload (no CPU leg).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 240 python3 $R/bench.py --steps 20 --warmup 3 --no-cpu > $R/gpurun_out/nn_cur.json 2> $R/gpurun_out/nn_cur.err || exit $?
echo ok
