#!/bin/bash
# GPU-box routine: the whole GPU suite, then C2 with the split-K fold on / off (interleaved A/B), and the
# 192-channel configs with their per-launch tables.
# usage (via gpurun): bash tools/r02_fold.sh <tag>
tag=$1
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $out/${tag}_test.log 2>&1 || exit $?
: > $out/${tag}_ab.log
for i in 1 2; do
  for v in 0 1; do
    CAI_SPLITK_FOLD_OFF=$v timeout -k 10 300 python bench.py --steps 50 --warmup 10 --cpu-seconds 0 --no-profile \
        >> $out/${tag}_ab.log 2>&1 || exit $?
    echo "fold_off=$v" >> $out/${tag}_ab.log
  done
done
: > $out/${tag}_models.log
for cfg in "bmshj2018-hyperprior 1 16" "cheng2020-attn 6 4" "bmshj2018-hyperprior 6 16" "mbt2018 1 16"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --model $1 --quality $2 --batch $3 --steps 20 --warmup 5 --cpu-seconds 0 \
      --ops-json $out/ops_${tag}_$1_q$2.json >> $out/${tag}_models.log 2>&1 || exit $?
done
