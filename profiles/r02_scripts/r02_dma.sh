#!/bin/bash
# GPU-box routine: conv parity on the DMA-footprint variant (lib/libcai_dma.so), then an interleaved C2 A/B
# (libcai.so vs libcai_dma.so) with per-launch tables.
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out
LIBDIR=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib
mkdir -p $out
cd $GRAFT_REPO_ROOT
CAI_LIB=$LIBDIR/libcai_dma.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q \
    -k "conv_fwd_bwd or act_chain or halo" --timeout 120 -p no:cacheprovider > $out/${tag}_test.log 2>&1 || exit $?
: > $out/${tag}_ab.log
for r in 1 2; do
  for v in libcai libcai_dma; do
    echo "== $v round $r" >> $out/${tag}_ab.log
    CAI_LIB=$LIBDIR/$v.so timeout -k 10 300 python bench.py --steps 50 --warmup 10 --cpu-seconds 0 \
        --ops-json $out/ops_${tag}_${v}_$r.json >> $out/${tag}_ab.log 2>&1 || exit $?
  done
done
