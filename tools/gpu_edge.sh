set -o pipefail
cd $GRAFT_REPO_ROOT
out=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $out
LIBDIR=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/edge_tests.log 2>&1 || exit $?
bash tools/kprof_ab_lib.sh edge libcai_base.so libcai.so || exit $?
bash tools/ab_env.sh edge 3 "CAI_LIB=$LIBDIR/libcai_base.so" "-"
