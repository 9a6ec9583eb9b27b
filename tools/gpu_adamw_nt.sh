#!/bin/bash
# AdamW non-temporal A/B (alternating processes on one box) + optimizer GPU tests.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "adam" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_adamw.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_adamw.log; [ $rc -eq 0 ] || exit $rc
for N in 1 0 1 0; do
  DLGM_ADAMW_NT=$N timeout -k 10 120 python tools/bench_kernels.py --only adamw > gpurun_out/adamw_nt$N.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/adamw_nt$N.json'));print('nt=$N', d['adamw_1G'])"
done
