#!/bin/bash
# kernel traces of short bench runs of C2' (hyperprior q6) and C3 (mbt2018-mean q1) for per-class step tables
cd /tmp && export TMPDIR=/tmp
out=$GRAFT_REPO_ROOT/gpurun_out
for cfg in "q6:--model bmshj2018-hyperprior --quality 6" "c3:--model mbt2018-mean --quality 1"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace -d $out/tr_$tag -o run --output-format csv -- \
      python3 $GRAFT_REPO_ROOT/bench.py $args --steps 6 --warmup 2 --cpu-seconds 0 --no-profile > $out/tr_$tag.log 2>&1 || exit 1
done
