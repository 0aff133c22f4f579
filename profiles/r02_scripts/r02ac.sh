cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_edge_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $o/r02ac_test.log 2>&1 || exit 1
: > $o/r02ac_bench.log
for s in 3 0 2 6 3 0 2 6; do
  CAI_EDGE_S2D_BPC=$s timeout -k 10 200 python bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-profile 2>/dev/null | python -c "import json,sys; print('bpc=$s', json.loads(sys.stdin.read())['value'])" >> $o/r02ac_bench.log || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r02ac_prof -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-profile > $GRAFT_REPO_ROOT/gpurun_out/r02ac_prof.log 2>&1
