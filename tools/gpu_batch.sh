#!/bin/bash
# GPU-box routine: optional pytest selection, then interleaved env A/B bench lines (tools/ab_env.sh).
# usage (via gpurun): GB_TESTS="tests/x.py -k y" bash tools/gpu_batch.sh <tag> <rounds> "<env A>" "<env B>" ...
tag=$1; rounds=$2; shift 2
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
cd $GRAFT_REPO_ROOT
if [ -n "$GB_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $GB_TESTS -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
      > $out/gb_${tag}_test.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $out/gb_${tag}_test.log; exit 1; }
  tail -3 $out/gb_${tag}_test.log
fi
bash tools/ab_env.sh $tag $rounds "$@" || exit 1
cat $out/ab_$tag.log
