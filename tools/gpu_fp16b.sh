#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_fp16_path.py tests/test_kernels_fp16_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fp16.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 4 --warmup 2 --dtype fp16 --n-layers 8 --no-telemetry > gpurun_out/bench_fp16_8l.json 2> gpurun_out/bench_fp16_8l.err &&
timeout -k 10 600 python bench.py --steps 6 --warmup 2 --dtype fp16 > gpurun_out/bench_fp16.json 2> gpurun_out/bench_fp16.err
