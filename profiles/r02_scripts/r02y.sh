cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $R/gpurun_out/r02y_p1 -o run --output-format csv -- python3 $R/tools/gdnbench.py > $R/gpurun_out/r02y_p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT -d $R/gpurun_out/r02y_p2 -o run --output-format csv -- python3 $R/tools/gdnbench.py > $R/gpurun_out/r02y_p2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE -d $R/gpurun_out/r02y_p3 -o run --output-format csv -- python3 $R/tools/gdnbench.py > $R/gpurun_out/r02y_p3.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r02y_t -o run --output-format csv -- python3 $R/tools/gdnbench.py > $R/gpurun_out/r02y_t.log 2>&1
