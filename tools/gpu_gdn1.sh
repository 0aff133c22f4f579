set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gdn_lane_gpu.py tests/test_gdn_gpu.py -x -q -k "gdn" --timeout 120 --timeout-method thread -p no:cacheprovider > $out/gdn1_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gdn or deferred" --timeout 120 --timeout-method thread -p no:cacheprovider >> $out/gdn1_tests.log 2>&1 || exit $?
bash tools/kprof_env.sh gdn1 "CAI_GDN_LANE=0" "-" || exit $?
bash tools/ab_env.sh gdn1 3 "CAI_GDN_LANE=0" "-"
