#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_gemm_mfma.py 8192 > gpurun_out/gemm_bench.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "permute or flash_attention" > gpurun_out/kern_test.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_engine_numerics.py -x -v --timeout 120 --timeout-method thread \
  -k "gpu or cuda" > gpurun_out/numerics_test.log 2>&1 &&
HIP_LAUNCH_BLOCKING=1 timeout -k 10 120 python -u tools/diag/groupk_steps.py > gpurun_out/groupk_run.log 2>&1
