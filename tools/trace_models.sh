#!/bin/bash
# kernel traces of short bench runs (C2, C5, C4) for per-class step tables (tools/step_classes.py)
cd /tmp && export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out
for cfg in "c2:--model bmshj2018-hyperprior --quality 1" "mm:--model multimodal" "c4:--model cheng2020-attn --quality 6 --batch 4"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace -d $out/tr_$tag -o run --output-format csv -- \
      python3 $GRAFT_REPO_ROOT/bench.py $args --steps 6 --warmup 2 --cpu-seconds 0 --no-profile > $out/tr_$tag.log 2>&1 || exit 1
done
