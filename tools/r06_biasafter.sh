#!/bin/bash
# r06 A/B: the halo weight gradient's bias sums behind each step's MFMAs (new) vs ahead of each fragment's (base = HEAD)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py tests/test_production_mix_gpu.py tests/test_bench_path_gpu.py > gpurun_out/ba_test.log 2>&1 || { tail -30 gpurun_out/ba_test.log; exit 1; }
tail -2 gpurun_out/ba_test.log
bash tools/kprof_libs.sh ba "wgrad_halo" "base new" $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-profile && cat gpurun_out/kl_ba.txt &&
bash tools/bench_ab.sh bac2 "base new" 3 && bash tools/bench_ab.sh bac4 "base new" 2 --model cheng2020-attn --quality 6 --batch 4 --steps 20 --warmup 5
