#!/bin/bash
# Attention tests after the fused-delta change, then the round-3 batch (NVMe offload_param test, 8B shadow, kernel stats).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "flash" -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_attn_r3i.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_attn_r3i.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r3f.sh
