set -e
out=gpurun_out; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "conv" -p no:cacheprovider > $out/ph_test.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --cpu-seconds 0 > $out/ph_bench_new.log 2>&1
CAI_HALO_PH_OFF=1 timeout -k 10 200 python bench.py --steps 50 --warmup 10 --cpu-seconds 0 > $out/ph_bench_off.log 2>&1
timeout -k 10 200 python bench.py --steps 50 --warmup 10 --cpu-seconds 0 > $out/ph_bench_new2.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/ph_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $GRAFT_REPO_ROOT/$out/ph_prof.log 2>&1
