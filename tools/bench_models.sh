#!/bin/bash
# GPU-box routine: one short bench line per model config (no CPU baseline), with each config's per-launch
# table (bench.py --ops-json) for the roofline / launch breakdown.
# usage (via gpurun): bash tools/bench_models.sh <tag>
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
: > $out/models_$tag.log
for cfg in "bmshj2018-factorized 1 16" "bmshj2018-hyperprior 1 16" "bmshj2018-hyperprior 6 16" \
           "mbt2018-mean 1 16" "mbt2018 1 16" "cheng2020-anchor 6 4" "cheng2020-attn 6 4" "multimodal 1 2"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --model $1 --quality $2 --batch $3 --steps 10 --warmup 3 --cpu-seconds 0 \
      --ops-json $out/ops_${tag}_$1_q$2.json >> $out/models_$tag.log 2>&1 \
      || { echo "FAILED $cfg rc=$?" >> $out/models_$tag.log; exit 1; }
done
