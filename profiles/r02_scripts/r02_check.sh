#!/bin/bash
# GPU-box routine (round 2): the new parity tests first, then the whole GPU suite, the default bench line with
# its per-launch table, and a rocprofv3 kernel-stats pass of a short bench.
# usage (via gpurun): bash tools/r02_check.sh <tag> [pytest -k expr]
tag=$1
kexpr=${2:-}
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
cd $GRAFT_REPO_ROOT
if [ -n "$kexpr" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -k "$kexpr" -s --timeout 300 --timeout-method thread \
      -p no:cacheprovider > $out/${tag}_test.log 2>&1 || exit $?
else
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -s --timeout 300 --timeout-method thread \
      -p no:cacheprovider > $out/${tag}_test.log 2>&1 || exit $?
fi
timeout -k 10 300 python bench.py --ops-json $out/${tag}_ops.json > $out/${tag}_bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/${tag}_prof -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-profile > $out/${tag}_prof.log 2>&1
