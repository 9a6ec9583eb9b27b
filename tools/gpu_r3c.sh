#!/bin/bash
# Targeted GPU check: grouped expert GEMMs, attention (ping-pong forward), kernel A/B, Mixtral expert strategies.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_mfma_gpu.py -k "grouped" -v --timeout 120 --timeout-method thread > gpurun_out/pytest_grouped.log 2>&1; rc=$?
tail -12 gpurun_out/pytest_grouped.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "flash" -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_attn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_kernels.py --only attn,attn_ab > gpurun_out/bench_kernels_attn.json 2> gpurun_out/bench_kernels_attn.err; rc=$?
cat gpurun_out/bench_kernels_attn.json; tail -3 gpurun_out/bench_kernels_attn.err; [ $rc -eq 0 ] || exit $rc
for MODE in torch 0 1; do
  DLGM_MOE_GROUPED=$MODE timeout -k 10 300 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 > gpurun_out/bench_mixtral_$MODE.json 2> gpurun_out/bench_mixtral_$MODE.err; rc=$?
  echo "MODE=$MODE"; cat gpurun_out/bench_mixtral_$MODE.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['value'],d['ms_per_step'],d['extra']['mfu_vs_2.5PF_dense_bf16'])"; tail -2 gpurun_out/bench_mixtral_$MODE.err; [ $rc -eq 0 ] || exit $rc
done
