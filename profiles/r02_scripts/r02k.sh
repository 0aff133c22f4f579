cd $GRAFT_REPO_ROOT
o=gpurun_out
: > $o/r02k_bench.log
for m in "bmshj2018-hyperprior 1 16" "mbt2018-mean 1 16" "mbt2018 1 16" "cheng2020-anchor 6 4"; do
  set -- $m
  for rep in 1 2 3; do
    for s in 0 1; do
      echo "$1 q$2 serial=$s" >> $o/r02k_bench.log
      CAI_HYPER_STREAM=$((1-s)) timeout -k 10 200 python bench.py --model $1 --quality $2 --batch $3 --steps 50 --warmup 5 --cpu-seconds 0 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])" >> $o/r02k_bench.log || exit 1
    done
  done
done
