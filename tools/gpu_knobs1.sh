set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out; mkdir -p $out
CAI_HALO_MIN_TILES=128 timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "conv_fwd_bwd" --timeout 120 --timeout-method thread -p no:cacheprovider > $out/knobs1_tests.log 2>&1 || exit $?
bash tools/kprof_env.sh knobs1 "-" "CAI_HALO_MIN_TILES=128" || exit $?
bash tools/ab_env.sh knobs1 3 "-" "CAI_HALO_MIN_TILES=128" "CAI_GDN_LANE_MIN_STEPS=1"
