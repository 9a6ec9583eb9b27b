#!/bin/bash
# Shadow-rank runs on one MI355X: rank 0 of the 8-GPU BASELINE configs 4 and 5 (per-rank HBM + compute time).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 420 python -u tools/shadow_rank.py --model llama3-70b --world 8 --ga 2 --steps 2 --warmup 1 --ckpt \
  --out gpurun_out/shadow_rank_llama3_70b_w8.json > gpurun_out/shadow_70b.log 2>&1 || { tail -20 gpurun_out/shadow_70b.log; exit 1; }
tail -3 gpurun_out/shadow_70b.log
timeout -k 10 300 python -u tools/shadow_rank.py --model mixtral-8x7b --world 8 --ep 8 --seq 4096 --ga 2 --steps 2 --warmup 1 --ckpt \
  --out gpurun_out/shadow_rank_mixtral_8x7b_ep8_w8.json > gpurun_out/shadow_mixtral.log 2>&1 || { tail -20 gpurun_out/shadow_mixtral.log; exit 1; }
tail -3 gpurun_out/shadow_mixtral.log
timeout -k 10 300 python -u tools/shadow_rank.py --model llama3-8b --world 8 --ga 4 --steps 2 --warmup 1 \
  --out gpurun_out/shadow_rank_llama3_8b_w8.json > gpurun_out/shadow_8b.log 2>&1 || { tail -20 gpurun_out/shadow_8b.log; exit 1; }
tail -3 gpurun_out/shadow_8b.log
