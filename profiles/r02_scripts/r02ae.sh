cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_edge_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $o/r02ae_test.log 2>&1 || exit 1
bash tools/kprof_libs.sh r02ae "edge_s2d" "base new x4pd2" $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-profile || exit 1
cd $GRAFT_REPO_ROOT
CAI_EDGE_S2D_BPC=2 bash tools/kprof_libs.sh r02ae_b2 "edge_s2d" "new x4pd2" $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-profile || exit 1
cd $GRAFT_REPO_ROOT
CAI_EDGE_S2D_BPC=0 bash tools/kprof_libs.sh r02ae_b0 "edge_s2d" "new" $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-profile || exit 1
