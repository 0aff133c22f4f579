#!/bin/bash
# r06: peak device memory (torch.cuda.max_memory_allocated over the bench run) and throughput with the deferred /
# batched weight gradients on (default) and off (CAI_WGRAD_BATCH=0), C2 / C4 / C5 -- ADVICE r05
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/wbm.log
: > $out
for cfg in "--model bmshj2018-hyperprior --quality 1" "--model cheng2020-attn --quality 6 --batch 4" "--model multimodal"; do
  for v in "CAI_WGRAD_BATCH=1" "CAI_WGRAD_BATCH=0"; do
    line=$(env $v timeout -k 10 300 python bench.py $cfg --steps 10 --warmup 3 --cpu-seconds 0 --no-profile 2>/dev/null | grep '^{') || exit 1
    echo "$cfg | $v | $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["unit"], "peak", d["max_memory_allocated_gb"], "GB")')" | tee -a $out
  done
done
