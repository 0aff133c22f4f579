#!/bin/bash
# GPU-box routine: per-kernel rocprofv3 stats of one bench run per environment setting (A/B of dispatch knobs),
# compared side by side with tools/kprof_cmp.py (first setting = base).
# usage (via gpurun): KP_ARGS="--model ..." bash tools/kprof_env.sh <tag> "<env A>" "<env B>"   ("-" = none)
tag=$1; shift
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
args=${KP_ARGS:-}
cd /tmp && export TMPDIR=/tmp
i=0
for v in "$@"; do
  envs=$v; [ "$v" = "-" ] && envs=""
  for kv in $envs; do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/kpe_${tag}_$i -o run --output-format csv -- \
      python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-profile $args > $out/kpe_${tag}_$i.log 2>&1 || exit $?
  for kv in $envs; do unset "${kv%%=*}"; done
  i=$((i+1))
done
python3 $GRAFT_REPO_ROOT/tools/kprof_cmp.py $out/kpe_${tag}_0 $out/kpe_${tag}_1 > $out/kpe_${tag}.txt
