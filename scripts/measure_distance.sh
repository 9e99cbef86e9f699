#!/bin/bash
# k_distance: parity tests, then bench_distance.py per variant ("NAME:ENV=VAL ...") for the
# full blimp and the reference's last submesh.  Stops at the first failure.
set -o pipefail
OUT=gpurun_out/dist
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_distance_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  for ag in all last; do
    env $envs timeout -k 10 200 python scripts/bench_distance.py --agent $ag --no-cpu > $OUT/${name}_$ag.log 2>&1 || { tail $OUT/${name}_$ag.log; exit 1; }
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], round(d['ms_per_step'],3), 'ms', round(d['value']/1e6,2), 'M poses/s fp64 frac', round(d['fp64']['frac'],4), d['work_per_step'])" $OUT/${name}_$ag.log "$name/$ag"
  done
done
