cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "gdn or models or golden or wide" --timeout 300 --timeout-method thread -p no:cacheprovider > $o/r02v_test.log 2>&1 || exit 1
: > $o/r02v_bench.log
for s in 0 1 0 1; do
  CAI_GDN_RING_OFF=$s timeout -k 10 200 python bench.py --steps 50 --warmup 5 --cpu-seconds 0 2>/dev/null | python -c "import json,sys; print('ring_off=$s', json.loads(sys.stdin.read())['value'])" >> $o/r02v_bench.log || exit 1
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --cpu-seconds 0 --ops-json $o/r02v_ops.json > /dev/null 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r02v_prof -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-profile > $GRAFT_REPO_ROOT/gpurun_out/r02v_prof.log 2>&1
