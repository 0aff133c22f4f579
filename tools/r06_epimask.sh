#!/bin/bash
# r06 A/B: the masked epilogue of the stride-1 input-gradient halo kernels -- direct from registers with every mask
# load ahead of the stores (new), staged through LDS with the aux chunks prefetched (lds), per-chunk loads (serial)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py tests/test_production_mix_gpu.py tests/test_models_gpu.py tests/test_resunit_gpu.py \
    > gpurun_out/em_test.log 2>&1 || { tail -30 gpurun_out/em_test.log; exit 1; }
tail -2 gpurun_out/em_test.log
bash tools/kprof_libs.sh em "conv_halo" "serial lds new" $GRAFT_REPO_ROOT/bench.py --model multimodal --steps 5 --warmup 2 --cpu-seconds 0 --no-profile && cat gpurun_out/kl_em.txt &&
bash tools/bench_ab.sh emmm "serial lds new" 2 --model multimodal --steps 10 --warmup 3 &&
bash tools/bench_ab.sh emc4 "serial lds new" 2 --model cheng2020-attn --quality 6 --batch 4 --steps 20 --warmup 5 &&
bash tools/bench_ab.sh emc2 "serial lds new" 2
