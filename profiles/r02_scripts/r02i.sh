cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "distributed or caller" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02i_test.log 2>&1
