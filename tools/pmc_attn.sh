# PMC counters for the attention kernels (separate run: --pmc with kernel-trace only, no sys/runtime trace).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/pmc/p1 -o run --output-format csv -- python3 tools/bench_kernels.py --only attn > gpurun_out/pmc/p1.log 2>&1
rc=$?; tail -3 gpurun_out/pmc/p1.log; exit $rc
