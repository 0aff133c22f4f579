#!/bin/bash
# r06 A/B: the Master decoder's aligner inputs fanned out (the cat hands its gradient slice to the patch embedding's
# dgrad epilogue) vs autograd's add (CAI_FANOUT=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_master_gpu.py tests/test_production_mix_gpu.py tests/test_distributed_gpu.py > gpurun_out/cf_test.log 2>&1 || { tail -30 gpurun_out/cf_test.log; exit 1; }
tail -2 gpurun_out/cf_test.log
AB_ARGS="--model multimodal --steps 10 --warmup 3 --cpu-seconds 0 --no-profile" bash tools/ab_env.sh cf 3 "CAI_FANOUT=0" "-" && cat gpurun_out/ab_cf.log
