#!/bin/bash
# k_distance at this head: bench lines (full blimp and the reference's last submesh, with the
# oracle's CPU rate) and a rocprofv3 kernel trace + stats of the full-blimp run.
export TMPDIR=/tmp
OUT=gpurun_out/dist_${TAG:-r17}
mkdir -p $OUT
set -o pipefail
timeout -k 10 300 python scripts/bench_distance.py --cpu-poses 100 > $OUT/bench_all.json 2> $OUT/bench_all.err || exit $?
timeout -k 10 300 python scripts/bench_distance.py --agent last --cpu-poses 300 > $OUT/bench_last.json 2> $OUT/bench_last.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 scripts/bench_distance.py --no-cpu > $OUT/kt.log 2>&1 || exit $?
find $OUT/kt -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
find $OUT/kt -name "run_kernel_trace.csv" -delete
grep k_distance $OUT/kernel_stats.csv | cut -d, -f1-5
