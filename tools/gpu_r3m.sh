#!/bin/bash
# Grouped MoE default: engine numerics + HIP-graph capture of the MoE loop, Mixtral EP8 shadow rank (expert W^T
# cache), Mixtral 2-layer bench eager and with HIP graphs.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_engine_numerics.py -k "mixtral or hip_graph" -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_moe_r3m.log 2>&1; rc=$?
tail -8 gpurun_out/pytest_moe_r3m.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/shadow_rank.py --model mixtral-8x7b --world 8 --ep 8 --seq 4096 --ga 2 --steps 2 --warmup 1 --ckpt \
  --out gpurun_out/shadow_rank_mixtral_8x7b_ep8_w8_r03.json > gpurun_out/shadow_mixtral_r03.log 2>&1; rc=$?
tail -2 gpurun_out/shadow_mixtral_r03.log; [ $rc -eq 0 ] || exit $rc
for G in "" "--hip-graphs"; do
  timeout -k 10 300 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 $G > gpurun_out/bench_mixtral_r3m$G.json 2> gpurun_out/bench_mixtral_r3m$G.err; rc=$?
  echo "graphs=$G"; python -c "import json;d=json.load(open('gpurun_out/bench_mixtral_r3m$G.json'));print(d['value'],d['ms_per_step'],d['extra']['mfu_vs_2.5PF_dense_bf16'],d['config'].get('hip_graphs'))"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_mixtral_r3m$G.err; exit $rc; }
done
