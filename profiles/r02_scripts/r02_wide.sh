#!/bin/bash
# GPU-box routine: the conv parity tests (incl. the halo stride-1 / 192-channel cases), then bench lines with
# per-launch tables for the 192-channel configs.
# usage (via gpurun): bash tools/r02_wide.sh <tag>
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "conv_fwd_bwd or act_chain" --timeout 120 \
    --timeout-method thread -p no:cacheprovider > $out/${tag}_test.log 2>&1 || exit $?
: > $out/${tag}_models.log
for cfg in "cheng2020-attn 6 4" "bmshj2018-hyperprior 6 16" "bmshj2018-hyperprior 1 16"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --model $1 --quality $2 --batch $3 --steps 10 --warmup 3 --cpu-seconds 0 \
      --ops-json $out/ops_${tag}_$1_q$2.json >> $out/${tag}_models.log 2>&1 || exit $?
done
