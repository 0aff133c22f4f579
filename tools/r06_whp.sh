L=$GRAFT_REPO_ROOT/165-learning-based-multi-modality-image-and-video-compression_amd/lib
cd $GRAFT_REPO_ROOT
CAI_LIB=$L/libcai_whpipe.so timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_bench_path_gpu.py -k "wgrad or halo or bench" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/whp_test.log 2>&1 || { tail -30 gpurun_out/whp_test.log; exit 1; }
tail -2 gpurun_out/whp_test.log
bash tools/kprof_libs.sh whp "wgrad_halo" "new whpipe whnob" $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-profile || exit 1
bash tools/kprof_libs.sh whp4 "wgrad_halo" "new whpipe" $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-profile --model cheng2020-attn --quality 6 --batch 4 || exit 1
cat gpurun_out/kl_whp.txt gpurun_out/kl_whp4.txt
bash tools/bench_ab.sh whp "new whpipe" 2
