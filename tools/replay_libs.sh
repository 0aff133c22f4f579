#!/bin/bash
# GPU-box routine: time one launch of the bench step (bench.py --roofline-only --replay) under each library
# variant, interleaved twice.  usage: bash tools/replay_libs.sh <tag> <kind:index> "<bench args>" <name...>
# (lib/libcai_<name>.so; "base" = lib/libcai.so)
tag=$1; rep=$2; bargs=$3; shift 3
out=$GRAFT_REPO_ROOT/gpurun_out
LIBDIR=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib
cd $GRAFT_REPO_ROOT
: > $out/rl_${tag}.log
for round in 1 2; do
  for v in "$@"; do
    if [ $v = base ]; then export CAI_LIB=$LIBDIR/libcai.so; else export CAI_LIB=$LIBDIR/libcai_$v.so; fi
    echo -n "$v " >> $out/rl_${tag}.log
    timeout -k 10 120 python bench.py --roofline-only --steps 50 --replay $rep $bargs 2>/dev/null \
        | grep '^{' >> $out/rl_${tag}.log || exit $?
  done
done
