#!/bin/bash
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
cd $GRAFT_REPO_ROOT
for cfg in "cheng2020-attn 6 4" "bmshj2018-hyperprior 6 16" "multimodal 1 2"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --model $1 --quality $2 --batch $3 --steps 10 --warmup 3 --cpu-seconds 0 \
      --ops-json $out/ops_r03a_$1_q$2.json >> $out/models_r03a.log 2>&1 || exit $?
done
