#!/bin/bash
# Grouped GEMM tests, then Mixtral 2-layer mode 1 kernel stats (grouped-M order + segmented dW) and the expert
# W^T cache A/B (mode 0 and 1 with DLGM_EXPERT_WT=1).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_mfma_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm_r3l.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gemm_r3l.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
DLGM_MOE_GROUPED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mix1b -o run --output-format csv -- python3 bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 2 --warmup 1 > gpurun_out/prof_mix1b.log 2>&1; rc=$?
tail -1 gpurun_out/prof_mix1b.log; [ $rc -eq 0 ] || exit $rc
for MODE in 0 1; do
  DLGM_EXPERT_WT=1 DLGM_MOE_GROUPED=$MODE timeout -k 10 300 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 > gpurun_out/bench_mixtral_r3l_wt_$MODE.json 2> gpurun_out/bench_mixtral_r3l_wt_$MODE.err; rc=$?
  echo "WT MODE=$MODE"; python -c "import json;d=json.load(open('gpurun_out/bench_mixtral_r3l_wt_$MODE.json'));print(d['value'],d['ms_per_step'],d['extra']['mfu_vs_2.5PF_dense_bf16'])"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_mixtral_r3l_wt_$MODE.err; exit $rc; }
done
