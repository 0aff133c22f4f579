#!/bin/bash
# GPU-box routine: per-kernel instruction-mix / stall counters over one probe program,
# one rocprofv3 --pmc pass per group (no tracing domains with --pmc).
# usage (via gpurun): bash tools/pmc_probe.sh <tag> <python script> [args...]
tag=$1; shift
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $out/pmcp_${tag}_$i -o run --output-format csv -- \
      python3 "$@" > $out/pmcp_${tag}_$i.log 2>&1
  rc=$?
  echo "group $i rc=$rc" >> $out/pmcp_${tag}.status
  if [ $rc -ge 124 ]; then exit $rc; fi
done
