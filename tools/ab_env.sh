#!/bin/bash
# GPU-box routine: the C2 bench line under several environment settings, each in its own process, the runs
# interleaved (A B C A B C ...) so box drift hits every variant alike.
# usage (via gpurun): bash tools/ab_env.sh <tag> <rounds> "<env settings A>" "<env settings B>" ...
# ("-" = no extra settings); bench flags come from $AB_ARGS (default: --steps 40 --warmup 10 --cpu-seconds 0
# --no-profile).  Writes gpurun_out/ab_<tag>.log: one "variant value ms" line per run.
tag=$1; rounds=$2; shift 2
out=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $out
args=${AB_ARGS:---steps 40 --warmup 10 --cpu-seconds 0 --no-profile}
: > $out/ab_$tag.log
for r in $(seq 1 $rounds); do
  for v in "$@"; do
    envs=$v; [ "$v" = "-" ] && envs=""
    line=$(env $envs timeout -k 10 240 python bench.py $args 2>>$out/ab_${tag}_err.log | tail -1) || { echo "FAILED $v" >> $out/ab_$tag.log; exit 1; }
    echo "$v $(echo "$line" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $out/ab_$tag.log
  done
done
