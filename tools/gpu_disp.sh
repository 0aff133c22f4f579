set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/disp_tests.log 2>&1 || exit $?
bash tools/ab_env.sh dispC2 3 "CAI_GLDS_M64=0" "-" || exit $?
AB_ARGS="--model bmshj2018-hyperprior --quality 6 --steps 20 --warmup 5 --cpu-seconds 0 --no-profile" bash tools/ab_env.sh dispC2p 2 "CAI_GLDS_M64=0" "-" || exit $?
AB_ARGS="--model cheng2020-attn --quality 6 --batch 4 --steps 10 --warmup 3 --cpu-seconds 0 --no-profile" bash tools/ab_env.sh dispC4 2 "CAI_GLDS_M64=0 CAI_SMALL_CONV_OFF=1" "-"
