cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "gdn or models or golden or kernels" --timeout 300 --timeout-method thread -p no:cacheprovider > $o/r02o_test.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --cpu-seconds 0 > $o/r02o_bench.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --quality 6 --steps 50 --warmup 5 --cpu-seconds 0 >> $o/r02o_bench.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r02o_prof -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-profile > $GRAFT_REPO_ROOT/gpurun_out/r02o_prof.log 2>&1
