#!/bin/bash
# Kernel check: the GPU numerics tests of the named kernels (-k expression) + their micro-benchmarks.
#   bash tools/gpu_kcheck.sh <pytest -k expr> <bench_kernels --only list>
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "$1" --timeout 120 --timeout-method thread > gpurun_out/pytest_k.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_kernels.py --only "$2" > gpurun_out/bench_k.json 2> gpurun_out/bench_k.err; rc=$?
cat gpurun_out/bench_k.json; exit $rc
