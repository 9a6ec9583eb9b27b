#!/bin/bash
# Closing validation at HEAD: full GPU suite + smoke, Mixtral 2-layer eager and HIP-graph captured.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
BENCH_STEPS=5 bash tools/gpu_round.sh test || exit 1
for G in "" "--hip-graphs"; do
  timeout -k 10 300 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 $G > gpurun_out/bench_mixtral_close$G.json 2> gpurun_out/bench_mixtral_close$G.err || { tail -10 gpurun_out/bench_mixtral_close$G.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_mixtral_close$G.json'));print('mixtral graphs=$G', d['value'],d['ms_per_step'],d['extra']['mfu_vs_2.5PF_dense_bf16'],d['config']['hip_graphs'])"
done
