#!/bin/bash
# GPU-box routine: interleaved bench.py lines of several library builds (lib/libcai_<name>.so; "new" =
# lib/libcai.so), N rounds.  usage (via gpurun): bash tools/bench_ab.sh <tag> "<libs>" [rounds] [bench args...]
tag=$1; libs=$2; rounds=${3:-2}; shift 3
out=$GRAFT_REPO_ROOT/gpurun_out
LIBDIR=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib
mkdir -p $out
cd $GRAFT_REPO_ROOT
for r in $(seq $rounds); do
  for v in $libs; do
    if [ $v = new ]; then export CAI_LIB=$LIBDIR/libcai.so; else export CAI_LIB=$LIBDIR/libcai_$v.so; fi
    line=$(timeout -k 10 200 python bench.py --steps 50 --warmup 10 --cpu-seconds 0 --no-profile "$@" 2>/dev/null | grep '^{') || exit 1
    echo "$v $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')" | tee -a $out/bab_$tag.log
  done
done
