cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu -k "models or golden or distributed or caller or master" --timeout 300 --timeout-method thread -p no:cacheprovider > $o/r02j_test.log 2>&1 || exit 1
for m in "bmshj2018-hyperprior 1" "bmshj2018-hyperprior 6" "mbt2018 1"; do
  set -- $m
  timeout -k 10 200 python bench.py --model $1 --quality $2 --steps 20 --warmup 5 --cpu-seconds 0 >> $o/r02j_bench.log 2>&1 || exit 1
  CAI_HYPER_STREAM=0 timeout -k 10 200 python bench.py --model $1 --quality $2 --steps 20 --warmup 5 --cpu-seconds 0 >> $o/r02j_bench.log 2>&1 || exit 1
done
