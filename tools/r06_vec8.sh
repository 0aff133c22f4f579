#!/bin/bash
# r06 A/B: 8-channel bf16 chunks for the channel aligner's affine and the Swin GELU (new) vs HEAD (base)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_master_gpu.py tests/test_production_mix_gpu.py > gpurun_out/v8_test.log 2>&1 || { tail -30 gpurun_out/v8_test.log; exit 1; }
tail -2 gpurun_out/v8_test.log
bash tools/kprof_libs.sh v8 "channel_affine|gelu" "base new" $GRAFT_REPO_ROOT/bench.py --model multimodal --steps 5 --warmup 2 --cpu-seconds 0 --no-profile && cat gpurun_out/kl_v8.txt &&
bash tools/bench_ab.sh v8mm "base new" 3 --model multimodal --steps 10 --warmup 3 && cat gpurun_out/bab_v8mm.log
