set -o pipefail
cd $GRAFT_REPO_ROOT
out=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $out
LIBDIR=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_models_wide_gpu.py -x -q -k "shuffle or cheng or attn or anchor" --timeout 200 --timeout-method thread -p no:cacheprovider > $out/shuf_tests.log 2>&1 || exit $?
KP_ARGS="--model cheng2020-attn --quality 6 --batch 4" bash tools/kprof_ab_lib.sh shuf libcai_base.so libcai.so || exit $?
AB_ARGS="--model cheng2020-attn --quality 6 --batch 4 --steps 10 --warmup 3 --cpu-seconds 0 --no-profile" bash tools/ab_env.sh shufc4 3 "CAI_LIB=$LIBDIR/libcai_base.so" "-"
