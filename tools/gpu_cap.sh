#!/bin/bash
# MoE capacity layout: GPU tests, Mixtral 2-layer bench grouped vs capacity (per-expert static-shape GEMMs).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_moe_capacity.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_cap.log 2>&1; rc=$?
tail -12 gpurun_out/pytest_cap.log; [ $rc -eq 0 ] || exit $rc
for M in 1 cap; do
  DLGM_MOE_GROUPED=$M timeout -k 10 300 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 > gpurun_out/bench_mixtral_$M.json 2> gpurun_out/bench_mixtral_$M.err; rc=$?
  echo "mode=$M"; [ $rc -eq 0 ] || { tail -15 gpurun_out/bench_mixtral_$M.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/bench_mixtral_$M.json'));print(d['value'],d['ms_per_step'],d['extra']['mfu_vs_2.5PF_dense_bf16'],d['extra']['peak_GiB_max_over_ranks'])"
done
timeout -k 10 240 python -u tools/diag/fill_sources.py > gpurun_out/fill_sources.log 2>&1; rc=$?
tail -25 gpurun_out/fill_sources.log; exit $rc
