#!/bin/bash
# GPU-box routine: average duration of kernels matching a pattern, for a python command run under each of
# several library builds (lib/libcai_<name>.so; "new" = lib/libcai.so).
# usage (via gpurun): bash tools/kprof_libs.sh <tag> <kernel-regex> "<libs>" <script.py> [args...]
tag=$1; pat=$2; libs=$3; shift 3
out=$GRAFT_REPO_ROOT/gpurun_out
LIBDIR=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
: > $out/kl_$tag.txt
for v in $libs; do
  if [ $v = new ]; then export CAI_LIB=$LIBDIR/libcai.so; else export CAI_LIB=$LIBDIR/libcai_$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kl_${tag}_$v -o run --output-format csv -- \
      python3 "$@" > $out/kl_${tag}_$v.log 2>&1 || exit $?
  python3 - "$out/kl_${tag}_$v" "$pat" "$v" >> $out/kl_$tag.txt <<'PY'
import csv, glob, re, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if re.search(sys.argv[2], r["Name"]):
        print(f"{sys.argv[3]:8s} calls {int(r['Calls']):5d} avg {float(r['AverageNs'])/1e3:9.2f} us min {float(r['MinNs'])/1e3:9.2f} | {r['Name'][:90]}")
PY
done
