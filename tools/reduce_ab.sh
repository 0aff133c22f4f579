#!/bin/bash
# GPU-box routine: the C2 step's batched reduce launch (tools/reduce_bench.py) under several library builds, then
# interleaved bench lines of the same builds.  usage (via gpurun): bash tools/reduce_ab.sh <tag> "<libs>" [rounds]
tag=$1; libs=$2; rounds=${3:-2}
out=$GRAFT_REPO_ROOT/gpurun_out
LIBDIR=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib
mkdir -p $out
cd $GRAFT_REPO_ROOT
: > $out/rab_$tag.log
for v in $libs; do
  if [ $v = new ]; then export CAI_LIB=$LIBDIR/libcai.so; else export CAI_LIB=$LIBDIR/libcai_$v.so; fi
  timeout -k 10 200 python tools/reduce_bench.py --tag $v >> $out/rab_$tag.log 2>&1 || exit 1
done
bash tools/bench_ab.sh $tag "$libs" $rounds || exit 1
cat $out/rab_$tag.log $out/bab_$tag.log
