#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of C5's 256->256 stride-1 halo launches (forward, input gradient, weight gradient),
# each replayed alone; one counter group per rocprofv3 run
out=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
for rep in conv_fwd:33 conv_dgrad:66 conv_wgrad:69; do
  t=c5_$(echo $rep | tr ':' '_')
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c -d $out/trf_${t}_$c -o run --output-format csv -- \
        python3 $GRAFT_REPO_ROOT/bench.py --model multimodal --roofline-only --steps 5 --replay $rep > $out/trf_${t}_$c.log 2>&1 || exit 1
  done
done
