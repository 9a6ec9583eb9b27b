#!/bin/bash
# MFMA GEMM + MoE permute + attention tail numerics, then the GEMM micro-bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_mfma_gpu.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/gemm_test.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "permute or flash_attention" > gpurun_out/kern_test.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_gemm_mfma.py 8192 > gpurun_out/gemm_bench.log 2>&1
