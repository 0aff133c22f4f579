#!/bin/bash
# r06 A/B: the N = 192 image-side weight gradient on the LDS-DMA ring (edge_wgrad_dma192_kernel) vs the general
# kernel (CAI_EDGE_WGRAD_DMA192=0): C2' (hyperprior q6) and mbt2018 q1
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_edge_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_models_wide_gpu.py \
    > gpurun_out/e192_test.log 2>&1 || { tail -30 gpurun_out/e192_test.log; exit 1; }
tail -2 gpurun_out/e192_test.log
KP_ARGS="--model bmshj2018-hyperprior --quality 6" bash tools/kprof_env.sh e192 "CAI_EDGE_WGRAD_DMA192=0" "-" || exit 1
grep -i "edge" gpurun_out/kpe_e192.txt
AB_ARGS="--model bmshj2018-hyperprior --quality 6 --steps 30 --warmup 5 --cpu-seconds 0 --no-profile" bash tools/ab_env.sh e192q6 3 "CAI_EDGE_WGRAD_DMA192=0" "-" && cat gpurun_out/ab_e192q6.log
AB_ARGS="--model mbt2018 --quality 1 --steps 30 --warmup 5 --cpu-seconds 0 --no-profile" bash tools/ab_env.sh e192mbt 2 "CAI_EDGE_WGRAD_DMA192=0" "-" && cat gpurun_out/ab_e192mbt.log
