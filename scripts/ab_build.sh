#!/bin/bash
# Usage: [OUTLIB=_lib_b] bash scripts/ab_build.sh <patch-file | git-rev>  (here, on the CPU)
# Builds a variant of libmpt.so -- the tree's csrc with a patch applied (or csrc as of a git
# revision) -- into motionplanningtoolkit_amd/$OUTLIB/libmpt.so, for scripts/ab_pair.sh (_lib_b)
# or scripts/ab_multi.sh (_lib_<name>).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUTLIB=${OUTLIB:-_lib_b}
W=/tmp/mpt_ab_src
rm -rf $W && mkdir -p $W/motionplanningtoolkit_amd
cp -r $R/include $W/include
if [ -f "$1" ]; then
  cp -r $R/motionplanningtoolkit_amd/csrc $W/motionplanningtoolkit_amd/csrc
  (cd $W && patch -p1 < "$(realpath $1)")
else
  (cd $R && git archive "$1" motionplanningtoolkit_amd/csrc include) | tar -x -C $W
fi
make -s -j8 -C $W/motionplanningtoolkit_amd/csrc OUT=$R/motionplanningtoolkit_amd/$OUTLIB $R/motionplanningtoolkit_amd/$OUTLIB/libmpt.so
ls -la $R/motionplanningtoolkit_amd/$OUTLIB/libmpt.so
