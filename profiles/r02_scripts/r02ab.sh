cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "conv" --timeout 300 --timeout-method thread -p no:cacheprovider > $o/r02ab_test.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r02ab_q6 -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --quality 6 --steps 10 --warmup 3 --cpu-seconds 0 --no-profile > $GRAFT_REPO_ROOT/gpurun_out/r02ab_q6.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r02ab_ch -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --model cheng2020-attn --quality 6 --batch 4 --steps 5 --warmup 2 --cpu-seconds 0 --no-profile > $GRAFT_REPO_ROOT/gpurun_out/r02ab_ch.log 2>&1
