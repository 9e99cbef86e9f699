#!/bin/bash
# SQ / TCC counter passes over a short bench (no CPU leg) for the instruction mix, stall
# picture and L2 hit rate of the kernels matching $KERNEL (a regex).  One pass per run
# (rocprofv3 does not split counters over passes).
#   KERNEL='k_grid_nn1_group|k_pairs' bash scripts/sq_profile.sh TAG
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-sq}
K=${KERNEL:-k_grid_nn1_group}
ARGS=${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu}
SCRIPT=${SCRIPT:-bench.py}  # e.g. SCRIPT=scripts/bench_distance.py BENCH_ARGS="--steps 2 --no-cpu"
mkdir -p $R/gpurun_out
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_IFETCH" \
           "TCC_HIT TCC_MISS TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "$K" --output-format csv -d $R/gpurun_out/prof_$TAG/p$i -o run -- python3 $R/$SCRIPT $ARGS > $R/gpurun_out/${TAG}_p$i.log 2>&1 || exit $?
done
echo done
