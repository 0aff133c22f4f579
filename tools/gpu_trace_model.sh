#!/bin/bash
# GPU-box routine: rocprofv3 kernel trace of one model config's graph-replayed bench steps (real in-step kernel times,
# unlike the per-launch ledger which times launches one at a time).  usage: bash tools/gpu_trace_model.sh <tag> <bench args>
tag=$1; shift
out=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/tr_$tag -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 --cpu-seconds 0 --no-profile "$@" > $out/tr_$tag.log 2>&1
