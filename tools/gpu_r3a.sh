#!/bin/bash
# Round-3 first GPU session: GPU tests, smoke, bf16 headline bench, fp16 bench (device-resident loss scaler).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?
tail -3 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 5 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 4 --warmup 2 --dtype fp16 > gpurun_out/bench_fp16.json 2> gpurun_out/bench_fp16.err; rc=$?
tail -3 gpurun_out/bench_fp16.err; cat gpurun_out/bench_fp16.json; exit $rc
