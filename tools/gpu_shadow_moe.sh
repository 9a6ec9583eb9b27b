#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u tools/shadow_rank.py --model mixtral-8x7b --world 8 --ep 8 --seq 4096 --ga 2 --steps 2 --warmup 1 --ckpt \
  --out gpurun_out/shadow_rank_mixtral_8x7b_ep8_w8.json > gpurun_out/shadow_mixtral.log 2>&1
rc=$?; tail -3 gpurun_out/shadow_mixtral.log; exit $rc
