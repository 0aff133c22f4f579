cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_noise_gpu.py tests/test_models_gpu.py tests/test_caller_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $o/r02aj_test.log 2>&1 || exit 1
: > $o/r02aj_bench.log
for v in old new old new; do
  if [ $v = old ]; then A="--keep-grads"; export CAI_TORCH_NOISE=1; else A=""; export CAI_TORCH_NOISE=0; fi
  echo -n "$v " >> $o/r02aj_bench.log
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 --cpu-seconds 0 --no-profile $A 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])" >> $o/r02aj_bench.log || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r02aj_prof -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-profile > $GRAFT_REPO_ROOT/gpurun_out/r02aj_prof.log 2>&1
