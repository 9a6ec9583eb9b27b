#!/bin/bash
# Llama-3-8B W=8 shadow rank, sync vs async collectives (peak memory and per-rank step time), plus the 70B layer.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for M in sync async; do
  FLAG=""; [ $M = async ] && FLAG="--async-comm"
  timeout -k 10 400 python tools/shadow_rank.py --model llama3-8b --world 8 --ga 4 --steps 2 --warmup 1 $FLAG --out gpurun_out/shadow_8b_w8_$M.json > gpurun_out/shadow_8b_w8_$M.log 2>&1; rc=$?
  tail -2 gpurun_out/shadow_8b_w8_$M.log; [ $rc -eq 0 ] || exit $rc
done
