#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench.py --steps 4 --warmup 2 --dtype fp16 --n-layers 8 --no-telemetry > gpurun_out/bench_fp16_8l.json 2> gpurun_out/bench_fp16_8l.err &&
timeout -k 10 300 python bench.py --steps 4 --warmup 2 --n-layers 8 --no-telemetry > gpurun_out/bench_bf16_8l.json 2> gpurun_out/bench_bf16_8l.err &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof16 -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --dtype fp16 --n-layers 8 --no-telemetry > gpurun_out/prof16.log 2>&1
