#!/bin/bash
# Bench variants (no CPU leg): per-round kernel times + collide work stats.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 240 python3 $R/bench.py --steps 10 --warmup 2 --no-cpu > $R/gpurun_out/diag_$tag.json 2> $R/gpurun_out/diag_$tag.err || exit $?
}
if [ -n "$BUCKETS" ]; then for b in $BUCKETS; do run b$b MPT_ENV_BUCKET=$b; done; else run ${TAG:-cur}; fi
echo ok
