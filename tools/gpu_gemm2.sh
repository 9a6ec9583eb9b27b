#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
HIP_LAUNCH_BLOCKING=1 timeout -k 10 120 python -u tools/diag/groupk_steps.py > gpurun_out/groupk_run.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gemm_mfma_gpu.py tests/test_engine_numerics.py -x -v --timeout 120 --timeout-method thread -k "gemm or dense or grouped or mixtral" > gpurun_out/gemm2_test.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_gemm_mfma.py 8192 > gpurun_out/gemm_bench2.log 2>&1 &&
DLGM_MOE_GROUPED=1 timeout -k 10 400 python -u bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 --no-telemetry > gpurun_out/bench_mixtral_grouped2.json 2> gpurun_out/bench_mixtral_grouped2.err
