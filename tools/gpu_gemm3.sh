#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/pmc
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_mfma_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gemm3_test.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_gemm_mfma.py 8192 > gpurun_out/gemm_bench3.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES -d gpurun_out/pmc/p3 -o run --output-format csv -- python3 tools/gemm_pmc_probe.py > gpurun_out/pmc/p3.log 2>&1
