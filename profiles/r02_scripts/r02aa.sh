cd $GRAFT_REPO_ROOT
o=gpurun_out
L=165-learning-based-multi-modality-image-and-video-compression_amd/lib
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "conv or models or golden" --timeout 300 --timeout-method thread -p no:cacheprovider > $o/r02aa_test.log 2>&1 || exit 1
: > $o/r02aa_bench.log
for v in libcai libcai_phold libcai libcai_phold; do
  CAI_LIB=$L/$v.so timeout -k 10 200 python bench.py --steps 50 --warmup 5 --cpu-seconds 0 2>/dev/null | python -c "import json,sys; print('$v', json.loads(sys.stdin.read())['value'])" >> $o/r02aa_bench.log || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r02aa_prof -o run --output-format csv -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-profile > $GRAFT_REPO_ROOT/gpurun_out/r02aa_prof.log 2>&1
