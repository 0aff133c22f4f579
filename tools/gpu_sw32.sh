set -o pipefail
cd $GRAFT_REPO_ROOT
out=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $out
LIBDIR=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_models_wide_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/sw32_tests.log 2>&1 || exit $?
AB_ARGS="--model cheng2020-attn --quality 6 --batch 4 --steps 10 --warmup 3 --cpu-seconds 0 --no-profile" bash tools/ab_env.sh sw32c4 2 "CAI_LIB=$LIBDIR/libcai_base.so" "-" || exit $?
AB_ARGS="--model cheng2020-anchor --quality 6 --batch 4 --steps 10 --warmup 3 --cpu-seconds 0 --no-profile" bash tools/ab_env.sh sw32c4a 2 "CAI_LIB=$LIBDIR/libcai_base.so" "-" || exit $?
bash tools/ab_env.sh sw32c2 2 "CAI_LIB=$LIBDIR/libcai_base.so" "-"
