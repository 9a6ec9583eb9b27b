#!/bin/bash
# Round 6: leased owner streams -- the full GPU suite, then the interleaved shadow reproducer.
set -o pipefail
mkdir -p gpurun_out/r06/suite
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/r06/suite/pytest_gpu_lease.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06/suite/pytest_gpu_lease.log | tail -6
[ $rc -le 1 ] || exit $rc
bash tools/diag/r06_stress.sh lease_async REPS=6
