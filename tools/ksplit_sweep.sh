#!/bin/bash
# GPU-box routine: bench lines under several split-K caps (CAI_KSPLIT_MAX).  usage: bash tools/ksplit_sweep.sh <tag>
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
cd $GRAFT_REPO_ROOT
: > $out/ks_$tag.log
for k in 0 1 2 4 8 0 2 4; do
  echo -n "cap=$k " >> $out/ks_$tag.log
  CAI_KSPLIT_MAX=$k timeout -k 10 200 python bench.py --steps 50 --warmup 10 --cpu-seconds 0 2>/dev/null | grep '^{' >> $out/ks_$tag.log || exit $?
done
