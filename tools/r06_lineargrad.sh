#!/bin/bash
# r06: Linear weights (viewed [out, in, 1, 1]) accumulate straight into the flat gradient buffer -- parity of the
# Swin / multimodal paths, C5 bench, and the kernel trace of the step's remaining ATen launches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_production_mix_gpu.py tests/test_master_gpu.py tests/test_models_gpu.py tests/test_distributed_gpu.py \
    > gpurun_out/lg_test.log 2>&1 || { tail -30 gpurun_out/lg_test.log; exit 1; }
tail -2 gpurun_out/lg_test.log
AB_ARGS="--model multimodal --steps 10 --warmup 3 --cpu-seconds 0 --no-profile" bash tools/ab_env.sh lg 2 "-" && cat gpurun_out/ab_lg.log
KP_ARGS="--model multimodal" bash tools/kprof_env.sh lg "-" "-"
