cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "gdn or bf16_bounds" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02f_test.log 2>&1 || exit $?
bash tools/replay_libs.sh gdn192 gdn_bwd:5 "--model bmshj2018-hyperprior --quality 6" base || exit $?
timeout -k 10 300 python bench.py --model bmshj2018-hyperprior --quality 6 --steps 20 --cpu-seconds 0 --ops-json gpurun_out/r02f_ops_q6.json > gpurun_out/r02f_bench.log 2>&1
