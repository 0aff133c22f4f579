#!/bin/bash
# r06 A/B: FanOutFn gradient joins in the 64 / 128-channel stride-1 halo input-gradient epilogues (new) vs a
# separate ATen add (base = HEAD)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py tests/test_production_mix_gpu.py tests/test_models_gpu.py \
    > gpurun_out/fo_test.log 2>&1 || { tail -30 gpurun_out/fo_test.log; exit 1; }
tail -2 gpurun_out/fo_test.log
bash tools/bench_ab.sh fomm "base new" 3 --model multimodal --steps 10 --warmup 3 && cat gpurun_out/bab_fomm.log
