#!/bin/bash
# Partial-tile quadrant skip in the grouped / dense MFMA GEMM: GPU tests, Mixtral 2-layer A/B (interleaved).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_moe_capacity.py tests/test_engine_numerics.py -m gpu -k "gemm or mfma or grouped or mixtral or kmajor or capacity" -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_qskip.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_qskip.log; [ $rc -eq 0 ] || exit $rc
for Q in 1 0 1 0; do
  DLGM_GEMM_QSKIP=$Q timeout -k 10 300 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 --no-telemetry > gpurun_out/bench_mixtral_q$Q.json 2> gpurun_out/bench_mixtral_q$Q.err; rc=$?
  [ $rc -eq 0 ] || { tail -15 gpurun_out/bench_mixtral_q$Q.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/bench_mixtral_q$Q.json'));print('qskip=$Q', d['value'],d['ms_per_step'],d['extra']['mfu_vs_2.5PF_dense_bf16'])"
done
