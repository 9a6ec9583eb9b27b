#!/bin/bash
# Kernel-time breakdowns (rocprofv3 kernel trace only): the Llama-3-8B headline step and the Mixtral-8x7B
# 2-layer step with the per-expert loop (mode 0) vs the grouped MFMA expert path (mode 1).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_llama -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --ga 2 > gpurun_out/prof_llama.log 2>&1; rc=$?
tail -2 gpurun_out/prof_llama.log; [ $rc -eq 0 ] || exit $rc
for MODE in 0 1; do
  DLGM_MOE_GROUPED=$MODE timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mix$MODE -o run --output-format csv -- python3 bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 2 --warmup 1 > gpurun_out/prof_mix$MODE.log 2>&1; rc=$?
  tail -2 gpurun_out/prof_mix$MODE.log; [ $rc -eq 0 ] || exit $rc
done
find gpurun_out/prof_llama gpurun_out/prof_mix0 gpurun_out/prof_mix1 -name "*kernel_stats*"
