#!/bin/bash
# A/B of config-5 bench lines: VAR="ENV=VAL ..." per variant, seeds from $SEEDS (default "32 256")
# Usage: TAG=x VARS="MPT_PT_NN_W=1;MPT_PT_NN_W=2" bash scripts/ab_c5.sh
set -e
TAG=${TAG:-ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
IFS=';' read -ra VS <<< "${VARS:-}"
for s in ${SEEDS:-32 256}; do
  for v in "${VS[@]}"; do
    name=$(echo "$v" | tr ' =' '__')
    env $v timeout -k 10 200 python bench.py --seeds $s --no-cpu > $OUT/c5_${s}_${name}.json 2>&1
    python3 -c "
import json
d=json.loads(open('$OUT/c5_${s}_${name}.json').read().strip().splitlines()[-1])
r=d['roofline']['stages']
print('$s $v', round(d['value']/1e6,2),'M', round(d['ms_per_step'],3),'ms', d['seeds_digest'][:16], {k:r[k]['ms'] for k in r})
" | tee -a $OUT/summary.txt
  done
done
