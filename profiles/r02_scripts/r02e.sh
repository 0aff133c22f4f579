cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "conv_fwd_bwd or halo" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02e_test.log 2>&1 || exit $?
bash tools/replay_libs.sh wg12 conv_wgrad:12 base && bash tools/replay_libs.sh wg1 conv_wgrad:1 base || exit $?
timeout -k 10 300 python bench.py --cpu-seconds 0 --ops-json gpurun_out/r02e_ops.json > gpurun_out/r02e_bench.log 2>&1
