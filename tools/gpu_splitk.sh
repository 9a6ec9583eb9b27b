#!/bin/bash
# Split-K narrow grouped-M GEMMs: GEMM tests, grouped probe and Mixtral 2-layer A/B (interleaved).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_mfma_gpu.py tests/test_moe_capacity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_splitk.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_splitk.log; [ $rc -eq 0 ] || exit $rc
for S in 1 0; do DLGM_GEMM_SPLITK=$S timeout -k 10 120 python3 tools/grouped_pmc_probe.py 2>/dev/null | sed "s/^/splitk=$S /" || exit 1; done
for S in 1 0 1 0; do
  DLGM_GEMM_SPLITK=$S timeout -k 10 300 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 --no-telemetry > gpurun_out/bench_mixtral_s$S.json 2> gpurun_out/bench_mixtral_s$S.err; rc=$?
  [ $rc -eq 0 ] || { tail -15 gpurun_out/bench_mixtral_s$S.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/bench_mixtral_s$S.json'));print('splitk=$S', d['value'],d['ms_per_step'],d['extra']['mfu_vs_2.5PF_dense_bf16'])"
done
