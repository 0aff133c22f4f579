#!/bin/bash
# GPU-box routine: the full GPU parity suite on the working tree's library, the durations of kernels matching
# a pattern under the HEAD (base, tools/build_base.sh) and working-tree (new) libraries, then interleaved
# bench lines.  usage (via gpurun): bash tools/ab.sh <tag> <kernel-regex>
tag=$1; pat=$2
out=$GRAFT_REPO_ROOT/gpurun_out
LIBDIR=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib
mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $out/ab_${tag}_test.log 2>&1 || exit $?
bash tools/kprof_libs.sh ab_$tag "$pat" "base new" $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 || exit $?
cd $GRAFT_REPO_ROOT
: > $out/ab_${tag}_bench.log
for v in base new base new; do
  if [ $v = new ]; then export CAI_LIB=$LIBDIR/libcai.so; else export CAI_LIB=$LIBDIR/libcai_base.so; fi
  echo -n "$v " >> $out/ab_${tag}_bench.log
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 --cpu-seconds 0 2>/dev/null | grep '^{' >> $out/ab_${tag}_bench.log || exit $?
done
