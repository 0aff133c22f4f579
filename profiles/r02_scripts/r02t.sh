cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $o/r02t_test.log 2>&1 || exit 1
: > $o/r02t_bench.log
for m in "bmshj2018-hyperprior 1 16" "bmshj2018-hyperprior 6 16" "mbt2018 1 16" "cheng2020-anchor 6 4"; do
  set -- $m
  timeout -k 10 200 python bench.py --model $1 --quality $2 --batch $3 --steps 50 --warmup 5 --cpu-seconds 0 2>/dev/null | python -c "import json,sys; print('$1 q$2', json.loads(sys.stdin.read())['value'])" >> $o/r02t_bench.log || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r02t_prof -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-profile > $GRAFT_REPO_ROOT/gpurun_out/r02t_prof.log 2>&1
