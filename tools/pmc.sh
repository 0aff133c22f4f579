#!/bin/bash
# GPU-box routine: HBM traffic of the bench's roofline kernel from two separate
# rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950;
# no tracing domains are combined with --pmc).
# usage (via gpurun): bash tools/pmc.sh <tag>
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d $out/pmc_${tag}_$c -o run --output-format csv -- \
      python3 $GRAFT_REPO_ROOT/bench.py --roofline-only --steps 20 > $out/pmc_${tag}_$c.log 2>&1 || exit $?
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $out/pmc_${tag}_FETCH_SIZE $out/pmc_${tag}_WRITE_SIZE \
    > $out/pmc_${tag}.json
