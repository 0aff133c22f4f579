#!/bin/bash
# GPU-box routine: parity tests, then a rocprofv3 kernel-trace of a short bench.
# usage (via gpurun): bash tools/gpu_check.sh <tag> [bench args...]
tag=$1; shift
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
timeout -k 10 600 python -m pytest tests -q -m gpu --timeout 300 -p no:cacheprovider > $out/test_$tag.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/test_$tag.log
if [ $rc -gt 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof_$tag -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --cpu-seconds 0 "$@" > $out/bench_$tag.log 2>&1
echo "prof rc=$?" >> $out/bench_$tag.log
