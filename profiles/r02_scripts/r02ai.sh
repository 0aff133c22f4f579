cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $o/r02ai_test.log 2>&1 || exit 1
bash tools/kprof_libs.sh r02ai "halo_kernel|halo_phase|edge_s2d" "ht0 new" $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-profile || exit 1
cd $GRAFT_REPO_ROOT
: > $o/r02ai_bench.log
for v in ht0 new ht0 new; do
  if [ $v = new ]; then export CAI_LIB=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib/libcai.so; else export CAI_LIB=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib/libcai_$v.so; fi
  echo -n "$v " >> $o/r02ai_bench.log
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 --cpu-seconds 0 --no-profile 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])" >> $o/r02ai_bench.log || exit 1
done
