#!/bin/bash
# A/B runs of bench.py on the GPU box: one bench line per variant, variants given as
# "NAME:ENV=VAL ENV2=VAL2" (env knobs such as MPT_NN1_XCD, MPT_PT_BBOX_PTS) or "NAME:" for
# the default, with the same bench arguments for all.  Each run has its own time limit; the
# script stops at the first failure.  Output: gpurun_out/ab_<tag>/<name>.json + .log.
#   BENCH_ARGS="--seeds 256 --steps 6 --warmup 3 --no-cpu" bash scripts/ab.sh c5 "base:" "bbox8k:MPT_PT_BBOX_PTS=8192"
TAG=$1; shift
ARGS=${BENCH_ARGS:---steps 20 --warmup 3 --no-cpu}
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
# a throw-away first run: the first bench process on a box ran a few % slow (clocks, caches)
if [ -z "$NO_WARM" ]; then
  timeout -k 10 300 python bench.py $ARGS > $OUT/warm.log 2>&1 || { tail -5 $OUT/warm.log; exit 1; }
fi
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  echo "== $name: $envs python bench.py $ARGS"
  env $envs timeout -k 10 300 python bench.py $ARGS > $OUT/$name.log 2>&1 || { tail -5 $OUT/$name.log; exit 1; }
  grep '^{' $OUT/$name.log > $OUT/$name.json
  python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d.get('kernel_ms_per_round') or {}; print(sys.argv[2], round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],3), 'ms/step', ' '.join('%s=%s' % kv for kv in k.items()))" $OUT/$name.json $name
done
