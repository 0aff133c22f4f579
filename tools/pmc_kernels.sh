#!/bin/bash
# GPU-box routine: per-kernel stall / LDS / cache counters over a short bench
# run, one rocprofv3 --pmc pass per counter group (no tracing domains with --pmc).
# usage (via gpurun): bash tools/pmc_kernels.sh <tag> [bench args...]
tag=$1; shift
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $out/pmck_${tag}_$i -o run --output-format csv -- \
      python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-graph "$@" > $out/pmck_${tag}_$i.log 2>&1
  rc=$?
  echo "group $i rc=$rc" >> $out/pmck_${tag}.status
  if [ $rc -ge 124 ]; then exit $rc; fi
done
