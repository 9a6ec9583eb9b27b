#!/bin/bash
# Round-3 batch: NVMe offload_param GPU test, 8B W=8 shadow sync vs async memory check, kernel-time breakdowns.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_runtime.py -k offload_param -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_offload_param.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_offload_param.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r3d.sh && bash tools/gpu_r3e.sh
