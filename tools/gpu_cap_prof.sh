#!/bin/bash
# Kernel stats of the Mixtral 2-layer bench in capacity mode (and the grouped default for reference).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for M in cap 1; do
  DLGM_MOE_GROUPED=$M timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_moe_$M -o run --output-format csv -- python3 bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 3 --warmup 1 --no-telemetry > gpurun_out/prof_moe_$M.log 2>&1 || { tail -20 gpurun_out/prof_moe_$M.log; exit 1; }
  tail -1 gpurun_out/prof_moe_$M.log
done
