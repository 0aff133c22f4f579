#!/bin/bash
# GPU-box routine: kernel traces of the one-graph fwd+bwd vs the phased exchange's graphs (tools/phase_times.py
# --only), C2 legacy plan; compared with tools/kprof_cmp.py.
out=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in plain phased; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $out/pt_$v -o run --output-format csv -- \
      python3 $GRAFT_REPO_ROOT/tools/phase_times.py --model bmshj2018-hyperprior --quality 1 --batch 16 --legacy --iters 20 --only $v > $out/pt_$v.log 2>&1 || exit 1
done
python3 $GRAFT_REPO_ROOT/tools/kprof_cmp.py $out/pt_plain $out/pt_phased
