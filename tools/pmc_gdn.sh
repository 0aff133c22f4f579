#!/bin/bash
# GPU-box routine: stall / LDS / HBM counters of the GDN kernels on the hyperprior's largest layer
# (tools/gdnbench.py), one rocprofv3 --pmc pass per counter group; summary with tools/pmc_kernels_summary.py.
# usage (via gpurun): bash tools/pmc_gdn.sh <tag>
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $out/pmck_${tag}_$i -o run --output-format csv -- \
      python3 $GRAFT_REPO_ROOT/tools/gdnbench.py > $out/pmck_${tag}_$i.log 2>&1
  rc=$?
  echo "group $i rc=$rc" >> $out/pmck_${tag}.status
  if [ $rc -ge 124 ]; then exit $rc; fi
done
python3 $GRAFT_REPO_ROOT/tools/pmc_kernels_summary.py $out/pmck_${tag} gdn > $out/pmck_${tag}.txt
