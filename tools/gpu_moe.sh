#!/bin/bash
# grouped GEMM numerics, device permute, Mixtral numerics, then the Mixtral 2-layer bench grouped vs per-expert
set -o pipefail
mkdir -p gpurun_out
HIP_LAUNCH_BLOCKING=1 timeout -k 10 120 python -u tools/diag/groupk_steps.py > gpurun_out/groupk_run.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gemm_mfma_gpu.py tests/test_kernels_gpu.py tests/test_engine_numerics.py \
  -x -v --timeout 120 --timeout-method thread -k "gemm or permute or moe or mixtral or grouped or dense" \
  > gpurun_out/moe_test.log 2>&1 &&
DLGM_MOE_GROUPED=1 timeout -k 10 400 python -u bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 \
  > gpurun_out/bench_mixtral_grouped.json 2> gpurun_out/bench_mixtral_grouped.err &&
DLGM_MOE_GROUPED=0 timeout -k 10 400 python -u bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 \
  --warmup 2 > gpurun_out/bench_mixtral_loop.json 2> gpurun_out/bench_mixtral_loop.err
