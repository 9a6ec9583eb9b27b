#!/bin/bash
# full GPU suite + smoke, headline bench (bf16), fp16 bench, kernel micro-bench
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 8 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 600 python bench.py --steps 4 --warmup 2 --dtype fp16 > gpurun_out/bench_fp16.json 2> gpurun_out/bench_fp16.err &&
timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/bench_kernels.json 2> gpurun_out/bench_kernels.err
