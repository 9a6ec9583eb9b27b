#!/bin/bash
# Grouped-M tile order (row tiles fastest within an expert): grouped GEMM tests, Mixtral 2-layer modes 0 / 1.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_mfma_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm_r3k.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gemm_r3k.log; [ $rc -eq 0 ] || exit $rc
for MODE in 0 1; do
  DLGM_MOE_GROUPED=$MODE timeout -k 10 300 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 > gpurun_out/bench_mixtral_r3k_$MODE.json 2> gpurun_out/bench_mixtral_r3k_$MODE.err; rc=$?
  echo "MODE=$MODE"; python -c "import json;d=json.load(open('gpurun_out/bench_mixtral_r3k_$MODE.json'));print(d['value'],d['ms_per_step'],d['extra']['mfu_vs_2.5PF_dense_bf16'])"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_mixtral_r3k_$MODE.err; exit $rc; }
done
