cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -k "conv or models or golden or master or halo" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02h_test.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --cpu-seconds 0 --ops-json gpurun_out/r02h_ops.json > gpurun_out/r02h_bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r02h_prof -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-profile > $GRAFT_REPO_ROOT/gpurun_out/r02h_prof.log 2>&1
