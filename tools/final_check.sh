#!/bin/bash
# GPU-box routine for a round's closing artefacts: full parity suite, smoke(), the default bench line (with
# CPU baseline), a rocprofv3 kernel-stats pass and the two PMC traffic passes of the roofline kernel.
# usage (via gpurun): bash tools/final_check.sh <tag>
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $out/fin_${tag}_test.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/fin_${tag}_smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $out/fin_${tag}_bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/fin_${tag}_prof -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $out/fin_${tag}_prof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && bash tools/pmc.sh fin_$tag
