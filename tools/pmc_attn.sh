#!/bin/bash
# PMC counters for the attention kernels: two passes (each within the per-block slot limits), kernel-trace
# only (no sys/runtime trace with --pmc on this pool). Output: gpurun_out/pmc/p{1,2}/run_counter_collection.csv
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/pmc/p1 -o run --output-format csv -- python3 tools/bench_kernels.py --only attn > gpurun_out/pmc/p1.log 2>&1 || { tail -5 gpurun_out/pmc/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmc/p2 -o run --output-format csv -- python3 tools/bench_kernels.py --only attn > gpurun_out/pmc/p2.log 2>&1 || { tail -5 gpurun_out/pmc/p2.log; exit 1; }
find gpurun_out/pmc -name "*.csv" | head
