#!/bin/bash
# GPU-box routine: per-kernel rocprofv3 stats of one bench run with the base and the new library.
# usage (via gpurun): bash tools/kprof_ab.sh <tag> [bench args...]
tag=$1; shift
out=$GRAFT_REPO_ROOT/gpurun_out
LIBDIR=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for v in base new; do
  if [ $v = base ]; then export CAI_LIB=$LIBDIR/libcai_base.so; else export CAI_LIB=$LIBDIR/libcai.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kp_${tag}_$v -o run --output-format csv -- \
      python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 "$@" > $out/kp_${tag}_$v.log 2>&1 || exit $?
done
python3 $GRAFT_REPO_ROOT/tools/kprof_cmp.py $out/kp_${tag}_base $out/kp_${tag}_new > $out/kp_${tag}.txt
