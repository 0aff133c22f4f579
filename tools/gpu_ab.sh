#!/bin/bash
# GPU-box routine: parity tests on the current libcai.so, then bench A/B of
# lib/libcai_base.so (previous build) vs lib/libcai.so, interleaved.
# usage (via gpurun): bash tools/gpu_ab.sh <tag> [bench args...]
tag=$1; shift
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
LIBDIR=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 -p no:cacheprovider > $out/test_$tag.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/test_$tag.log
if [ $rc -gt 1 ]; then exit $rc; fi
: > $out/ab_$tag.log
for r in 1 2; do
  for v in base new; do
    if [ $v = base ]; then L=$LIBDIR/libcai_base.so; else L=$LIBDIR/libcai.so; fi
    echo "== $v round $r" >> $out/ab_$tag.log
    CAI_LIB=$L timeout -k 10 300 python bench.py --cpu-seconds 0 "$@" >> $out/ab_$tag.log 2>&1 || exit $?
  done
done
