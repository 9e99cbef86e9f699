#!/bin/bash
# One rocprofv3 kernel trace of config 5 at 30 timed rounds (the run that ended in a host
# segmentation fault in round 1, before the per-joint-stream state and the reserved joint
# sort buffers): kernel stats + the tail of the log, whatever the outcome.
export TMPDIR=/tmp
OUT=gpurun_out/c5_30
mkdir -p $OUT
ulimit -c 0
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 bench.py --seeds 256 --steps 30 --warmup 3 --no-cpu > $OUT/run.log 2>&1
rc=$?
echo "rc=$rc" | tee $OUT/rc.txt
tail -c 2000 $OUT/run.log
rm -f $OUT/kt/run_kernel_trace.csv
exit 0
