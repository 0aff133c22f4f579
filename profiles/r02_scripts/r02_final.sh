#!/bin/bash
# GPU-box routine for the closing artefacts of a session: full parity suite, smoke(), the default bench line
# (with the CPU baseline), a rocprofv3 kernel-stats pass of a short bench, and the per-config lines.
# usage (via gpurun): bash tools/r02_final.sh <tag>
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $out/fin_${tag}_test.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/fin_${tag}_smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --ops-json $out/fin_${tag}_ops.json > $out/fin_${tag}_bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/fin_${tag}_prof -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-profile > $out/fin_${tag}_prof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && bash tools/bench_models.sh fin_$tag
