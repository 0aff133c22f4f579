set -o pipefail
cd $GRAFT_REPO_ROOT
out=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
CAI_REDUCE_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/rsplit -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-profile > $out/rsplit.log 2>&1
