#!/bin/bash
# Usage: TAG=x bash scripts/ab_multi.sh "<legs>" <variant>...  (on the GPU box)
# A = this tree's libmpt.so; each variant V = motionplanningtoolkit_amd/_lib_V/libmpt.so (built by
# scripts/ab_build.sh with OUTLIB=_lib_V) run from a copy of the tree.  Rounds A, V1, V2, ...,
# twice, each leg set by scripts/ab_legs.sh into gpurun_out/${TAG}_<name><rep>/.
TAG=${TAG:?set TAG}
LEGS=$1; shift
R=$(pwd)
for v in "$@"; do
  B=/tmp/mpt_ab_$v
  rm -rf $B && mkdir -p $B
  tar -C $R --exclude=./gpurun_out -cf - . | tar -C $B -xf - || exit 1
  cp $R/motionplanningtoolkit_amd/_lib_$v/libmpt.so $B/motionplanningtoolkit_amd/_lib/libmpt.so || exit 1
done
for rep in 1 2; do
  TAG=${TAG}_A$rep bash scripts/ab_legs.sh $LEGS || exit 1
  for v in "$@"; do
    (cd /tmp/mpt_ab_$v && TAG=${TAG}_$v$rep bash scripts/ab_legs.sh $LEGS) || exit 1
    cp -r /tmp/mpt_ab_$v/gpurun_out/${TAG}_$v$rep $R/gpurun_out/ || exit 1
  done
done
echo ab_multi done
