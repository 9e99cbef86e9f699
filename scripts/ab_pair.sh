#!/bin/bash
# Usage: TAG=x bash scripts/ab_pair.sh [legs...]  (on the GPU box)
# A = this tree's libmpt.so, B = motionplanningtoolkit_amd/_lib_b/libmpt.so (scripts/ab_build.sh)
# in a copy of the tree; the legs (scripts/ab_legs.sh) run A, B, A, B on the same box.
TAG=${TAG:?set TAG}
R=$(pwd)
B=/tmp/mpt_ab_b
rm -rf $B && mkdir -p $B
tar -C $R --exclude=./gpurun_out -cf - . | tar -C $B -xf - || exit 1
cp $R/motionplanningtoolkit_amd/_lib_b/libmpt.so $B/motionplanningtoolkit_amd/_lib/libmpt.so || exit 1
for rep in 1 2; do
  TAG=${TAG}_A$rep bash scripts/ab_legs.sh "$@" || exit 1
  (cd $B && TAG=${TAG}_B$rep bash scripts/ab_legs.sh "$@") || exit 1
  cp -r $B/gpurun_out/${TAG}_B$rep $R/gpurun_out/ || exit 1
done
echo ab_pair done
