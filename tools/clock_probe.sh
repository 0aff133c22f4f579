#!/bin/bash
# GPU-box routine: effective shader clock per kernel (GRBM_GUI_ACTIVE / 8 / duration) for several library
# builds (MI355X_MICROARCH.md, DVFS give-back).  usage: bash tools/clock_probe.sh <tag> "<libs>" <script> [args]
tag=$1; libs=$2; shift 2
out=$GRAFT_REPO_ROOT/gpurun_out
LIBDIR=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for v in $libs; do
  if [ $v = new ]; then export CAI_LIB=$LIBDIR/libcai.so; else export CAI_LIB=$LIBDIR/libcai_$v.so; fi
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace -d $out/clk_${tag}_$v -o run --output-format csv -- \
      python3 "$@" > $out/clk_${tag}_$v.log 2>&1 || exit $?
done
