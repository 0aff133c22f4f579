#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
AB_ARGS="--model cheng2020-attn --quality 6 --batch 4 --steps 20 --warmup 5 --cpu-seconds 0 --no-profile" bash tools/ab_env.sh c4k 3 "-" "CAI_WG_BLOCKS_R192=64" "CAI_WG_BLOCKS_R192=96" "CAI_RW_SPLITS=16" && cat gpurun_out/ab_c4k.log
