#!/bin/bash
# Mixtral-8x7B (2 layers, seq 4096) throughput at several micro-batch / GA shapes (one box, one process each)
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
IFS=, read -ra CFGS <<< "${MOE_CFGS:-1 4,2 4,4 4,2 8,1 16}"
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  timeout -k 10 400 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --mbs $1 --ga $2 --steps 4 --warmup 2 --no-telemetry > gpurun_out/moe_m$1_g$2.json 2> gpurun_out/moe_m$1_g$2.err || { tail -5 gpurun_out/moe_m$1_g$2.err; exit 1; }
  echo "mbs=$1 ga=$2 $(python3 -c "import json;d=json.load(open('gpurun_out/moe_m$1_g$2.json'));print(d['value'], d['ms_per_step'], d['extra']['mfu_vs_2.5PF_dense_bf16'], d['extra']['mem']['peak_GiB'])")"
done
