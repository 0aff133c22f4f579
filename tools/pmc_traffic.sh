# GPU-box routine: FETCH_SIZE / WRITE_SIZE passes (one counter group per rocprofv3 run) of replayed launches
# of the C2 step; the counter outputs land in gpurun_out/trf_<kind>_<index>_{f,w}; record them on the host
# with tools/pmc_traffic_update.py.  usage: bash tools/pmc_traffic.sh kind:index [kind:index ...]
out=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
for rep in "$@"; do
  t=$(echo $rep | tr ':' '_')
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $out/trf_${t}_f -o run --output-format csv -- \
      python3 $GRAFT_REPO_ROOT/bench.py --roofline-only --steps 10 --replay $rep > $out/trf_${t}_f.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $out/trf_${t}_w -o run --output-format csv -- \
      python3 $GRAFT_REPO_ROOT/bench.py --roofline-only --steps 10 --replay $rep > $out/trf_${t}_w.log 2>&1 || exit 1
done
