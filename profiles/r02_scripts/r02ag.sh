cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_edge_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $o/r02ag_test.log 2>&1 || exit 1
CAI_LIB=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib/libcai_gspd2.so timeout -k 10 900 python -u -m pytest tests/test_edge_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $o/r02ag_test2.log 2>&1 || exit 1
bash tools/kprof_libs.sh r02ag "edge_s2d" "new gs nt gsnt gspd2" $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-profile || exit 1
cd $GRAFT_REPO_ROOT
: > $o/r02ag_bench.log
for v in new gs new gs; do
  if [ $v = new ]; then export CAI_LIB=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib/libcai.so; else export CAI_LIB=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib/libcai_$v.so; fi
  echo -n "$v " >> $o/r02ag_bench.log
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 --cpu-seconds 0 --no-profile 2>/dev/null | python -c "import json,sys; print(json.loads(sys.stdin.read())['value'])" >> $o/r02ag_bench.log || exit 1
done
