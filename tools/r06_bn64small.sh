#!/bin/bash
# r06 A/B: 64-channel stride-1 halo tiles on small maps with wider outputs (CAI_HALO_S1_BN64_SMALL) -- C4, C3', C5
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py tests/test_production_mix_gpu.py tests/test_models_gpu.py tests/test_resunit_gpu.py \
    > gpurun_out/b64s_test.log 2>&1 || { tail -30 gpurun_out/b64s_test.log; exit 1; }
tail -2 gpurun_out/b64s_test.log
KP_ARGS="--model cheng2020-attn --quality 6 --batch 4" bash tools/kprof_env.sh b64s "CAI_HALO_S1_BN64_SMALL=0" "-" || exit 1
head -16 gpurun_out/kpe_b64s.txt
AB_ARGS="--model cheng2020-attn --quality 6 --batch 4 --steps 20 --warmup 5 --cpu-seconds 0 --no-profile" bash tools/ab_env.sh b64s 3 "CAI_HALO_S1_BN64_SMALL=0" "-" && cat gpurun_out/ab_b64s.log
AB_ARGS="--model cheng2020-anchor --quality 6 --batch 4 --steps 20 --warmup 5 --cpu-seconds 0 --no-profile" bash tools/ab_env.sh b64sa 2 "CAI_HALO_S1_BN64_SMALL=0" "-" && cat gpurun_out/ab_b64sa.log
