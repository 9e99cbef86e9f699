#!/bin/bash
# SQ counters of the incremental index's new-point sort (config 5, 32 seeds)
export TMPDIR=/tmp
mkdir -p gpurun_out/${SQTAG:-sqsort}
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "${KREGEX:-k_pt_inc_sort}" --output-format csv -d gpurun_out/${SQTAG:-sqsort}/p$i -o run -- python3 bench.py --seeds 32 --steps 3 --warmup 5 --no-cpu > gpurun_out/${SQTAG:-sqsort}/p$i.log 2>&1 || exit $?
done
python3 scripts/sq_summary.py gpurun_out/${SQTAG:-sqsort} > gpurun_out/${SQTAG:-sqsort}/summary.txt
