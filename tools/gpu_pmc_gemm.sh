#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d gpurun_out/pmc/p1 -o run --output-format csv -- python3 tools/gemm_pmc_probe.py > gpurun_out/pmc/p1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_INSTS_VMEM -d gpurun_out/pmc/p2 -o run --output-format csv -- python3 tools/gemm_pmc_probe.py > gpurun_out/pmc/p2.log 2>&1
