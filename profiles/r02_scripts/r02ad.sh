cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_edge_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $o/r02ad_test.log 2>&1 || exit 1
bash tools/kprof_libs.sh r02ad "edge_s2d" "base new pd2 nost nold" $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-profile || exit 1
cd $GRAFT_REPO_ROOT
for b in 2 4 6; do
  CAI_EDGE_S2D_BPC=$b bash tools/kprof_libs.sh r02ad_b$b "edge_s2d" "new pd2" $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-profile || exit 1
  cd $GRAFT_REPO_ROOT
done
