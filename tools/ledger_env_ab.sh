#!/bin/bash
# GPU-box routine: per-launch ledgers of one model config under several env settings (A/B of dispatch knobs).
# usage (via gpurun): bash tools/ledger_env_ab.sh <tag> <model> <quality> <batch> "ENV1=.. ENV2=.." ["..." ...]
tag=$1; model=$2; q=$3; b=$4; shift 4
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
cd $GRAFT_REPO_ROOT
i=0
for envs in "-" "$@"; do
  e=""; [ "$envs" != "-" ] && e="$envs"
  echo "== $envs" >> $out/envab_$tag.log
  env $e timeout -k 10 300 python bench.py --model $model --quality $q --batch $b --steps 10 --warmup 3 \
      --cpu-seconds 0 --ops-json $out/envab_${tag}_$i.json >> $out/envab_$tag.log 2>&1 || exit $?
  i=$((i+1))
done
