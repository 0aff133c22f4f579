#!/bin/bash
# GPU-box routine: per-kernel rocprofv3 stats of one C2 bench run per library build (A/B of compile-time variants
# built by tools/build_variants.sh), compared with tools/kprof_cmp.py (first = base).
# usage (via gpurun): [KP_ARGS="..."] bash tools/kprof_ab_lib.sh <tag> <libA.so> <libB.so>
tag=$1; la=$2; lb=$3
out=$GRAFT_REPO_ROOT/gpurun_out
LIBDIR=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
i=0
for l in $la $lb; do
  CAI_LIB=$LIBDIR/$l timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kpl_${tag}_$i -o run --output-format csv -- \
      python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-profile ${KP_ARGS:-} > $out/kpl_${tag}_$i.log 2>&1 || exit $?
  i=$((i+1))
done
python3 $GRAFT_REPO_ROOT/tools/kprof_cmp.py $out/kpl_${tag}_0 $out/kpl_${tag}_1 > $out/kpl_${tag}.txt
