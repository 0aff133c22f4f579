cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -k "models or golden or coding or master or pack" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02g_test.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --cpu-seconds 0 --ops-json gpurun_out/r02g_ops.json > gpurun_out/r02g_bench.log 2>&1
