#!/bin/bash
# GPU-box routine: the GPU parity tests on the working tree's library, the durations of kernels matching a
# pattern under a base and the working-tree (new) library, then interleaved bench lines.
# usage (via gpurun): bash tools/ab.sh <tag> <kernel-regex>
#   AB_BASE   base library name: lib/libcai_<AB_BASE>.so (default "base": tools/build_base.sh builds it from HEAD)
#   AB_TESTS  pytest arguments (default: the whole GPU suite, "tests -m gpu"; "-" skips the tests)
#   AB_BENCH  extra bench.py arguments for the profiled run and the bench lines (e.g. "--model bmshj2018-factorized")
tag=$1; pat=$2
base=${AB_BASE:-base}
tests=${AB_TESTS:-tests -m gpu}
out=$GRAFT_REPO_ROOT/gpurun_out
LIBDIR=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib
mkdir -p $out
cd $GRAFT_REPO_ROOT
if [ "$tests" != "-" ]; then
  timeout -k 10 900 python -u -m pytest $tests -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
      > $out/ab_${tag}_test.log 2>&1 || exit $?
fi
bash tools/kprof_libs.sh ab_$tag "$pat" "$base new" $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 \
    $AB_BENCH || exit $?
cd $GRAFT_REPO_ROOT
: > $out/ab_${tag}_bench.log
for v in $base new $base new; do
  if [ $v = new ]; then export CAI_LIB=$LIBDIR/libcai.so; else export CAI_LIB=$LIBDIR/libcai_$v.so; fi
  echo -n "$v " >> $out/ab_${tag}_bench.log
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 --cpu-seconds 0 --no-profile $AB_BENCH 2>/dev/null \
      | grep '^{' >> $out/ab_${tag}_bench.log || exit $?
done
