cd $GRAFT_REPO_ROOT
o=gpurun_out
L=165-learning-based-multi-modality-image-and-video-compression_amd/lib
: > $o/r02z_bench.log
for v in libcai libcai_pad16 libcai_pad48 libcai libcai_pad16 libcai_pad48; do
  CAI_LIB=$L/$v.so timeout -k 10 200 python bench.py --steps 50 --warmup 5 --cpu-seconds 0 2>/dev/null | python -c "import json,sys; print('$v', json.loads(sys.stdin.read())['value'])" >> $o/r02z_bench.log || exit 1
done
