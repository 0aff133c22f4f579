#!/bin/bash
# GPU-box routine: the quad-kernel parity test and tools/quad_bench.py under several library builds
# (lib/libcai_<name>.so; "new" = lib/libcai.so), bench lines interleaved twice.
# usage (via gpurun): bash tools/quad_ab.sh <tag> "<libs>"
tag=$1; libs=$2
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
LIBDIR=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib
mkdir -p $out
cd $GRAFT_REPO_ROOT
for v in $libs; do
  if [ $v = new ]; then export CAI_LIB=$LIBDIR/libcai.so; else export CAI_LIB=$LIBDIR/libcai_$v.so; fi
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
      tests/test_kernels_gpu.py -k quad > $out/test_$v.log 2>&1 || { echo "test $v failed"; exit 1; }
done
for r in 1 2; do
  for v in $libs; do
    if [ $v = new ]; then export CAI_LIB=$LIBDIR/libcai.so; else export CAI_LIB=$LIBDIR/libcai_$v.so; fi
    timeout -k 10 120 python tools/quad_bench.py --tag $v >> $out/bench.log 2>&1 || exit 1
  done
done
cat $out/bench.log
