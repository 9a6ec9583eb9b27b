#!/bin/bash
# Grouped-K chunk remap: GEMM/MoE GPU tests, Mixtral A/B (DLGM_GEMM_CHUNK_REMAP toggles grouped-K chunks AND the
# grouped-M balanced remap), kernel stats.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_moe_capacity.py tests/test_gemm_mfma_gpu.py tests/test_engine_numerics.py -k "mixtral or pad_plan or kmajor or capacity or hip_graph or grouped" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_kchunk.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_kchunk.log; [ $rc -eq 0 ] || exit $rc
for C in 1 0 1 0; do
  DLGM_GEMM_CHUNK_REMAP=$C timeout -k 10 300 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 --no-telemetry > gpurun_out/bench_mixtral_kc$C.json 2> gpurun_out/bench_mixtral_kc$C.err; rc=$?
  [ $rc -eq 0 ] || { tail -15 gpurun_out/bench_mixtral_kc$C.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/bench_mixtral_kc$C.json'));print('chunk=$C', d['value'],d['ms_per_step'],d['extra']['mfu_vs_2.5PF_dense_bf16'])"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_moe_kc -o run --output-format csv -- python3 bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 3 --warmup 1 --no-telemetry > gpurun_out/prof_moe_kc.log 2>&1 || { tail -20 gpurun_out/prof_moe_kc.log; exit 1; }
