#!/bin/bash
# Round 6: shadow-mesh heap pooling -- the interleaved asynchronous reproducer, then the full GPU suite.
set -o pipefail
mkdir -p gpurun_out/r06/stress gpurun_out/r06/suite
export HSA_ENABLE_IPC_MODE_LEGACY=0
REPS=8 timeout -k 10 300 python -u tools/diag/r06_shadow_stress.py > gpurun_out/r06/stress/pool_async2.log 2>&1
rc=$?; echo "pool_async rc=$rc"; grep -E "async_mismatches" gpurun_out/r06/stress/pool_async2.log | grep -v '"env"' \
    | python3 -c "import sys,json; d={k: v['async_mismatches'] for l in sys.stdin for k, v in json.loads(l).items()}; print(sum(d.values()), d)"
[ $rc -eq 0 ] && ! grep -q "HSA_STATUS_ERROR" gpurun_out/r06/stress/pool_async2.log || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/r06/suite/pytest_gpu_pool.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r06/suite/pytest_gpu_pool.log | tail -8
exit $rc
