cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in ${CSORT_VARIANTS:-1 0}; do
MPT_PT_CSORT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3w_prof$v -o run -- python3 bench.py --seeds ${SEEDS:-32} --no-cpu --no-variants > gpurun_out/r3w_prof$v.log 2>&1 || exit 1
f=$(find gpurun_out/r3w_prof$v -name "*kernel_stats.csv" | head -1); echo "CSORT=$v"; grep -E "inc_(sort|csort|crank|merge|ncodes|npos|boxes|top)" $f | cut -d, -f1-8
done
