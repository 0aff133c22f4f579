set -o pipefail
cd $GRAFT_REPO_ROOT
out=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_models_wide_gpu.py -x -q -k "residual or cheng or attn or anchor" --timeout 200 --timeout-method thread -p no:cacheprovider > $out/res_tests.log 2>&1 || exit $?
KP_ARGS="--model cheng2020-attn --quality 6 --batch 4" bash tools/kprof_env.sh res "CAI_RESIDUAL_FUSE=0" "-" || exit $?
AB_ARGS="--model cheng2020-attn --quality 6 --batch 4 --steps 10 --warmup 3 --cpu-seconds 0 --no-profile" bash tools/ab_env.sh resc4 3 "CAI_RESIDUAL_FUSE=0" "-"
