#!/bin/bash
# Round 6: the zero3_offload_param shadow-async mismatch of the validation batch -- the pinned-memory-aware stream
# audit over the shadow-async suite, the new audit self-test, and the two runtime tests changed after that batch.
set -o pipefail
mkdir -p gpurun_out/r06/offload
export HSA_ENABLE_IPC_MODE_LEGACY=0
P="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 400 $P tests/test_stream_audit.py tests/test_gpu_runtime.py -m gpu \
  > gpurun_out/r06/offload/runtime.log 2>&1; echo "runtime rc=$?"; tail -3 gpurun_out/r06/offload/runtime.log
DLGM_STREAM_AUDIT=1 timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread \
  tests/test_shadow_async_gpu.py -m gpu > gpurun_out/r06/offload/shadow_audit.log 2>&1
echo "shadow_audit rc=$?"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06/offload/shadow_audit.log | tail -8
