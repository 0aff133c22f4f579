#!/bin/bash
# GPU-box routine: conv parity tests on the working tree's library, then the halo kernels' durations under the
# HEAD (base) and working-tree (new) libraries, then interleaved bench lines.
# usage (via gpurun): bash tools/halo_ab.sh <tag>
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out
LIBDIR=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib
mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread \
    -k "conv" -p no:cacheprovider > $out/hab_${tag}_test.log 2>&1 || exit $?
bash tools/kprof_libs.sh hab_$tag "conv_halo" "base new" $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 || exit $?
cd $GRAFT_REPO_ROOT
: > $out/hab_${tag}_bench.log
for v in base new base new; do
  if [ $v = new ]; then export CAI_LIB=$LIBDIR/libcai.so; else export CAI_LIB=$LIBDIR/libcai_base.so; fi
  echo -n "$v " >> $out/hab_${tag}_bench.log
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 --cpu-seconds 0 2>/dev/null | grep '^{' >> $out/hab_${tag}_bench.log || exit $?
done
