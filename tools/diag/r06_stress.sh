#!/bin/bash
# Round 6: async-vs-sync shadow mismatch frequency after the suite's preceding GPU tests ran in the same process.
set -o pipefail
mkdir -p gpurun_out/r06/stress
export HSA_ENABLE_IPC_MODE_LEGACY=0
HISTORY=1 REPS=${REPS:-30} timeout -k 10 700 python -u tools/diag/r06_shadow_stress.py > gpurun_out/r06/stress/history.log 2>&1
echo "history rc=$?"; grep -E "threads_after|async_mismatches" gpurun_out/r06/stress/history.log | cut -c1-1500
