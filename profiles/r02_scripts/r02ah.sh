cd $GRAFT_REPO_ROOT
bash tools/kprof_libs.sh r02ah "edge_s2d" "gs gsnost gsnold" $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-profile || exit 1
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/membench.py > gpurun_out/r02ah_mem.log 2>&1
