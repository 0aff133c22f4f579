cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $o/r02m_test.log 2>&1 || exit 1
: > $o/r02m_bench.log
for m in "bmshj2018-hyperprior 1 16" "bmshj2018-hyperprior 6 16" "mbt2018 1 16" "cheng2020-anchor 6 4"; do
  set -- $m
  for rep in 1 2; do
    for s in 1 0; do
      echo "$1 q$2 wgrad_stream=$s" >> $o/r02m_bench.log
      CAI_WGRAD_STREAM=$s timeout -k 10 200 python bench.py --model $1 --quality $2 --batch $3 --steps 50 --warmup 5 --cpu-seconds 0 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])" >> $o/r02m_bench.log || exit 1
    done
  done
done
