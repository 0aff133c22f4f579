set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "conv_fwd_bwd or cheng2020" --timeout 120 --timeout-method thread -p no:cacheprovider > $out/m64_tests.log 2>&1 || exit $?
bash tools/ledger_env_ab.sh m64 cheng2020-attn 6 4 "CAI_GLDS_M64=0" "CAI_SMALL_CONV_OFF=1" "CAI_SMALL_WGRAD_OFF=1" || exit $?
AB_ARGS="--model cheng2020-attn --quality 6 --batch 4 --steps 10 --warmup 3 --cpu-seconds 0 --no-profile" bash tools/ab_env.sh m64 2 "CAI_GLDS_M64=0" "-"
