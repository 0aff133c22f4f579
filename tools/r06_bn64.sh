#!/bin/bash
# r06 A/B: 64-channel stride-1 halo tiles (CAI_HALO_S1_BN64) and 64-row k3 weight-gradient tiles
# (CAI_HALO_WGRAD_K3_ROWS64) on C5 multimodal
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py tests/test_production_mix_gpu.py tests/test_models_gpu.py \
    > gpurun_out/bn64_test.log 2>&1 || { tail -30 gpurun_out/bn64_test.log; exit 1; }
tail -2 gpurun_out/bn64_test.log
KP_ARGS="--model multimodal" bash tools/kprof_env.sh bn64 "CAI_HALO_S1_BN64=0 CAI_HALO_WGRAD_K3_ROWS64=0" "-" || exit 1
cat gpurun_out/kpe_bn64.txt | head -30
AB_ARGS="--model multimodal --steps 10 --warmup 3 --cpu-seconds 0 --no-profile" bash tools/ab_env.sh bn64 2 \
    "CAI_HALO_S1_BN64=0 CAI_HALO_WGRAD_K3_ROWS64=0" "CAI_HALO_WGRAD_K3_ROWS64=0" "CAI_HALO_S1_BN64=0" "-" && cat gpurun_out/ab_bn64.log
