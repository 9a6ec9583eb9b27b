#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_kernels_fp16_gpu.py tests/test_engine_numerics.py -x -v --timeout 200 --timeout-method thread -k "flash or attention or chunked or llama" > gpurun_out/attn2_test.log 2>&1 &&
DLGM_ATTN_BWD_STREAMS=0 timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/bench_kernels_1s.json 2> gpurun_out/bench_kernels_1s.err &&
DLGM_ATTN_BWD_STREAMS=1 timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/bench_kernels_2s.json 2> gpurun_out/bench_kernels_2s.err &&
timeout -k 10 600 python bench.py --steps 6 --warmup 2 --no-telemetry > gpurun_out/bench_2s.json 2> gpurun_out/bench_2s.err &&
DLGM_ATTN_BWD_STREAMS=0 timeout -k 10 600 python bench.py --steps 6 --warmup 2 --no-telemetry > gpurun_out/bench_1s.json 2> gpurun_out/bench_1s.err
