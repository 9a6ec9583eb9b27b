#!/bin/bash
# Round 6: the full GPU suite (one process), log under gpurun_out/r06/suite/.
set -o pipefail
mkdir -p gpurun_out/r06/suite
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/r06/suite/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06/suite/pytest_gpu.log | tail -8
exit $rc
