#!/bin/bash
# round record: full GPU suite + smoke + headline bench + kernel stats profile
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2c -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-telemetry > gpurun_out/prof_r2c.log 2>&1
