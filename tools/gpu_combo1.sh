set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_phhalf.sh || exit $?
bash tools/kprof_ab_lib.sh fwd2 libcai.so libcai_fwd2.so || exit $?
bash tools/pmc_kernels.sh c2a
