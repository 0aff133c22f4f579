#!/bin/bash
# GPU-box routine: PMC counters of ONE launch of the bench step, replayed alone (bench.py --roofline-only
# --replay kind:index), one rocprofv3 --pmc pass per counter group (no tracing domains with --pmc).
# Summaries: python tools/pmc_kernels_summary.py gpurun_out/pmcr_<tag> <kernel substring>
# usage (via gpurun): bash tools/pmc_replay.sh <tag> <kind:index|dominant> [bench args...]
tag=$1; rep=$2; shift 2
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
ra=""
if [ "$rep" != "dominant" ]; then ra="--replay $rep"; fi
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $out/pmcr_${tag}_$i -o run --output-format csv -- \
      python3 $GRAFT_REPO_ROOT/bench.py --roofline-only --steps 10 $ra "$@" > $out/pmcr_${tag}_$i.log 2>&1
  rc=$?
  echo "group $i rc=$rc" >> $out/pmcr_${tag}.status
  if [ $rc -ne 0 ]; then exit $rc; fi
done
