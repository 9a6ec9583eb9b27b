#!/bin/bash
# Fused expert gradient statistics (grouped-K dW epilogue): GPU tests, then Mixtral 2-layer A/B, alternating.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_mfma_gpu.py tests/test_moe_capacity.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_xstats.log 2>&1; rc=$?
tail -1 gpurun_out/pytest_xstats.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_xstats.log | head -20; exit $rc; }
for N in ${XS_ORDER:-1 0 1 0}; do
  DLGM_FUSED_XSTATS=$N timeout -k 10 300 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 > gpurun_out/bench_xstats$N.json 2> gpurun_out/bench_xstats$N.err || { tail -10 gpurun_out/bench_xstats$N.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_xstats$N.json'));print('xstats=$N', d['value'],d['ms_per_step'],d['extra'].get('final_loss'),d['extra'].get('final_grad_norm'))"
done
