#!/bin/bash
# r06 A/B: the LDS-DMA weight gradient bias sums behind the MFMAs (new) vs ahead (base = HEAD)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py tests/test_production_mix_gpu.py tests/test_bench_path_gpu.py > gpurun_out/bg_test.log 2>&1 || { tail -30 gpurun_out/bg_test.log; exit 1; }
tail -2 gpurun_out/bg_test.log
bash tools/kprof_libs.sh bg "wgrad_glds" "base new" $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-profile && cat gpurun_out/kl_bg.txt &&
bash tools/bench_ab.sh bgc2 "base new" 3 && bash tools/bench_ab.sh bgc4 "base new" 2 --model cheng2020-attn --quality 6 --batch 4 --steps 20 --warmup 5
