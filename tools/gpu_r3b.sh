#!/bin/bash
# Round-3 GPU session: GPU tests (incl. async shadow + ping-pong forward), smoke, kernel A/B, bf16 and fp16 bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?
tail -3 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_kernels.py --only attn,attn_ab > gpurun_out/bench_kernels_attn.json 2> gpurun_out/bench_kernels_attn.err; rc=$?
cat gpurun_out/bench_kernels_attn.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 5 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 4 --warmup 2 --dtype fp16 > gpurun_out/bench_fp16.json 2> gpurun_out/bench_fp16.err; rc=$?
tail -3 gpurun_out/bench_fp16.err; cat gpurun_out/bench_fp16.json; exit $rc
