cd $GRAFT_REPO_ROOT
o=gpurun_out
timeout -k 10 120 python tools/membench.py > $o/r02p_mem.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r02p_prof -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/tools/membench.py > $GRAFT_REPO_ROOT/gpurun_out/r02p_prof.log 2>&1
