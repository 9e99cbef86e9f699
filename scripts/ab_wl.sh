#!/bin/bash
# A/B of the single-tree workloads' bench lines (config 2, blimp-room, snake): VARS="ENV=VAL ...;..."
# Usage: TAG=x VARS="MPT_X=0" bash scripts/ab_wl.sh
set -e
TAG=${TAG:-abwl}
OUT=gpurun_out/$TAG
mkdir -p $OUT
IFS=';' read -ra VS <<< "${VARS:-MPT_X=0}"
for wl in ${WORKLOADS:-blimp blimp-room snake}; do
  for v in "${VS[@]}"; do
    name=$(echo "$v" | tr ' =' '__')
    env $v timeout -k 10 200 python bench.py --workload $wl --no-cpu --no-variants > $OUT/${wl}_${name}.json 2>&1
    python3 -c "
import json
d=json.loads(open('$OUT/${wl}_${name}.json').read().strip().splitlines()[-1])
r=d['roofline']['stages']
print('$wl $v', round(d['value']/1e6,2),'M', round(d['ms_per_step'],4),'ms', {k:r[k]['ms'] for k in r})
" | tee -a $OUT/summary.txt
  done
done
