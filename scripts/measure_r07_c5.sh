#!/bin/bash
# Config 5 (256 seeds) bench lines at the rounds of the committed profile (profiles/r07/c5:
# rocprofv3 of --steps 6 --warmup 3; the seeds' trees, and so the joint NN launch's work, grow
# with every round), three repeats (run-to-run spread of the 32-stream schedule).
OUT=gpurun_out/m16
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --seeds 256 --steps 6 --warmup 3 --no-cpu > $OUT/c5_$i.log 2>&1 || exit $?
  grep '^{' $OUT/c5_$i.log > $OUT/bench_c5_$i.json
done
echo all done
