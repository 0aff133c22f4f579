cd $GRAFT_REPO_ROOT
o=gpurun_out
: > $o/r02n_bench.log
for cap in 0 1 2 4 8; do
  for m in "bmshj2018-hyperprior 1 16" "mbt2018 1 16"; do
    set -- $m
    echo "$1 q$2 ksplit_max=$cap" >> $o/r02n_bench.log
    CAI_KSPLIT_MAX=$cap timeout -k 10 200 python bench.py --model $1 --quality $2 --batch $3 --steps 50 --warmup 5 --cpu-seconds 0 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])" >> $o/r02n_bench.log || exit 1
  done
done
