#!/bin/bash
# GPU-box routine: parity tests, then an interleaved bench A/B.
# Variants are environment settings: AB_BASE / AB_NEW (e.g. "CAI_GDN_TWO_PASS=1"),
# default: lib/libcai_base.so vs lib/libcai.so.
# usage (via gpurun): [AB_BASE=... AB_NEW=...] bash tools/gpu_ab.sh <tag> [bench args...]
tag=$1; shift
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
LIBDIR=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib
BASE=${AB_BASE:-CAI_LIB=$LIBDIR/libcai_base.so}
NEW=${AB_NEW:-CAI_LIB=$LIBDIR/libcai.so}
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 -p no:cacheprovider > $out/test_$tag.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/test_$tag.log
if [ $rc -gt 1 ]; then exit $rc; fi
: > $out/ab_$tag.log
for r in 1 2; do
  for v in base new; do
    if [ $v = base ]; then E=$BASE; else E=$NEW; fi
    echo "== $v ($E) round $r" >> $out/ab_$tag.log
    env $E timeout -k 10 300 python bench.py --cpu-seconds 0 "$@" >> $out/ab_$tag.log 2>&1 || exit $?
  done
done
