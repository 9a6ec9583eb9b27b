#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_engine_numerics.py -x -v --timeout 120 --timeout-method thread -k "mixtral" > gpurun_out/moe3_test.log 2>&1 &&
for d in auto off; do
timeout -k 10 400 python -u bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 --no-telemetry --defer-expert-wgrad $d > gpurun_out/bench_mixtral_defer_$d.json 2> gpurun_out/bench_mixtral_defer_$d.err || exit 1
done &&
timeout -k 10 500 python -u bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 16 --steps 3 --warmup 1 --no-telemetry > gpurun_out/bench_mixtral_ga16.json 2> gpurun_out/bench_mixtral_ga16.err
