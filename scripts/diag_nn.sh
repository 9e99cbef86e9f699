#!/bin/bash
# NN variants on the bench workload (no CPU leg).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 240 python3 $R/bench.py --steps 10 --warmup 2 --no-cpu > $R/gpurun_out/nn_sort.json 2> $R/gpurun_out/nn_sort.err || exit $?
MPT_NN_NOSORT=1 timeout -k 10 240 python3 $R/bench.py --steps 10 --warmup 2 --no-cpu > $R/gpurun_out/nn_nosort.json 2> $R/gpurun_out/nn_nosort.err || exit $?
echo ok
