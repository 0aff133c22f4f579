cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "wgrad or models or golden or conv or gdn" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02d_test.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --cpu-seconds 0 --ops-json gpurun_out/r02d_ops.json > gpurun_out/r02d_bench.log 2>&1 || exit $?
bash tools/pmc_replay.sh wg12 conv_wgrad:12 && bash tools/pmc_replay.sh ph12 conv_dgrad:12 && bash tools/pmc_replay.sh gdn5 gdn_bwd:5
