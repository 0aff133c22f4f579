set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out; mkdir -p $out
CAI_HALO_PH_HALF=1 timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/phhalf_tests.log 2>&1 || exit $?
bash tools/kprof_env.sh phhalf "-" "CAI_HALO_PH_HALF=1" || exit $?
bash tools/ab_env.sh phhalf 3 "-" "CAI_HALO_PH_HALF=1"
