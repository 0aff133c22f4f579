#!/bin/bash
# GPU-box routine: rocprofv3 counter passes (one group per pass) over tools/quad_bench.py, then a per-kernel
# summary (tools/pmc_kernels_summary.py).  usage (via gpurun): bash tools/quad_pmc.sh <tag> [quad_bench args...]
tag=$1; shift
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_BUSY_CYCLES" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $out/p$i -o run --output-format csv -- \
      python3 $GRAFT_REPO_ROOT/tools/quad_bench.py --iters 20 "$@" > $out/p$i.log 2>&1
  rc=$?
  echo "group $i rc=$rc" >> $out/status
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 - $out <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    if "quad" not in k and "phase" not in k:
        continue
    print(k)
    for c, xs in sorted(v.items()):
        print(f"   {c:28s} {sum(xs) / len(xs):16.1f}  (n={len(xs)})")
PY
