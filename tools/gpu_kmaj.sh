#!/bin/bash
# K-contiguous deferred grouped dW: GPU tests, Mixtral 2-layer bench with and without it.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_moe_capacity.py tests/test_engine_numerics.py -k "mixtral or pad_plan or kmajor or capacity or hip_graph" -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_kmaj.log 2>&1; rc=$?
tail -6 gpurun_out/pytest_kmaj.log; [ $rc -eq 0 ] || exit $rc
for K in 1 0; do
  DLGM_MOE_KMAJOR_DW=$K timeout -k 10 300 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 > gpurun_out/bench_mixtral_k$K.json 2> gpurun_out/bench_mixtral_k$K.err; rc=$?
  echo "kmajor=$K"; [ $rc -eq 0 ] || { tail -15 gpurun_out/bench_mixtral_k$K.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/bench_mixtral_k$K.json'));print(d['value'],d['ms_per_step'],d['extra']['mfu_vs_2.5PF_dense_bf16'],d['extra']['peak_GiB_max_over_ranks'])"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_moe_k1 -o run --output-format csv -- python3 bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 3 --warmup 1 --no-telemetry > gpurun_out/prof_moe_k1.log 2>&1 || { tail -20 gpurun_out/prof_moe_k1.log; exit 1; }
