#!/bin/bash
# r06: C4 latent-layer dispatch A/B (conv_small on big-K small-M layers vs split-K; wgrad_small on/off)
set -o pipefail
cd $GRAFT_REPO_ROOT
C4="--model cheng2020-attn --quality 6 --batch 4"
KP_ARGS="$C4" bash tools/kprof_env.sh c4s "-" "CAI_SMALL_CONV_KMAX512=4096" "CAI_SMALL_CONV_OFF=1" "CAI_SMALL_WGRAD_OFF=1" || exit 1
for i in 0 1 2 3; do python3 tools/trace_step.py gpurun_out/kpe_c4s_$i/run_kernel_trace.csv > gpurun_out/kpe_c4s_${i}_step.txt || exit 1; done
AB_ARGS="$C4 --steps 20 --warmup 5 --cpu-seconds 0 --no-profile" bash tools/ab_env.sh c4s 2 "-" "CAI_SMALL_CONV_KMAX512=4096" "CAI_SMALL_CONV_OFF=1" "CAI_SMALL_WGRAD_OFF=1"
cat gpurun_out/ab_c4s.log
