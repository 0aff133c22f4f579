#!/bin/bash
# r06 A/B: the one-rank step captured as ONE graph (default) vs two graphs (--two-graphs), interleaved
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/og.log
: > $out
for r in 1 2 3; do
  for cfg in "--model bmshj2018-hyperprior --quality 1 --steps 50 --warmup 10" "--model cheng2020-attn --quality 6 --batch 4 --steps 20 --warmup 5"; do
    for v in "" "--two-graphs"; do
      line=$(timeout -k 10 300 python bench.py $cfg $v --cpu-seconds 0 --no-profile 2>/dev/null | grep '^{') || exit 1
      echo "$cfg $v | $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')" | tee -a $out
    done
  done
done
