#!/bin/bash
# GPU-box routine: parity tests, a plain bench line, then a rocprofv3
# kernel-trace of a short bench (the profiler inflates tiny kernels ~4x, so
# the plain line is the throughput number).
# usage (via gpurun): bash tools/gpu_check.sh <tag> [bench args...]
tag=$1; shift
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
timeout -k 10 600 python -m pytest tests -q -m gpu --timeout 300 -p no:cacheprovider > $out/test_$tag.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/test_$tag.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py "$@" > $out/bench_$tag.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof_$tag -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --cpu-seconds 0 "$@" > $out/bench_prof_$tag.log 2>&1
echo "prof rc=$?" >> $out/bench_prof_$tag.log
