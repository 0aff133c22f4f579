cd /tmp && export TMPDIR=/tmp
for s in 0 1; do
CAI_HYPER_STREAM=$s timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r02l_prof$s -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --model mbt2018 --steps 10 --warmup 3 --cpu-seconds 0 --no-profile > $GRAFT_REPO_ROOT/gpurun_out/r02l_prof$s.log 2>&1 || exit 1
done
