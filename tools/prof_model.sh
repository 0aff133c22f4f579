#!/bin/bash
# GPU-box routine: rocprofv3 kernel trace of a short bench of one model config.
# usage (via gpurun): bash tools/prof_model.sh <tag> <model> <quality> <batch>
tag=$1; model=$2; q=$3; b=$4
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof_$tag -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --model $model --quality $q --batch $b --steps 10 --warmup 3 --cpu-seconds 0 \
    > $out/bench_prof_$tag.log 2>&1
echo "prof rc=$?" >> $out/bench_prof_$tag.log
