#!/bin/bash
# Tune the Llama-3-8B GEMMs through hipBLASLt (tools/bench_gemm_lt.py --write), bring the table back,
# then A/B the headline bench with the tuned table on / off / on.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/tuned
timeout -k 10 900 python -u tools/bench_gemm_lt.py --all --write "$@" > gpurun_out/gemm_lt.log 2>&1; rc=$?
cut -c1-300 gpurun_out/gemm_lt.log; [ $rc -eq 0 ] || exit $rc
cp distributed_llm_training_gpu_manager_amd/tuned/gemm_lt_v*.json gpurun_out/tuned/
for v in 1 0 1; do
  DLGM_GEMM_LT=$v timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_lt$v.json 2> gpurun_out/bench_lt$v.err; rc=$?
  echo "lt=$v $(python -c "import json;d=json.load(open('gpurun_out/bench_lt$v.json'));print(d['value'],d['ms_per_step'])")"
  [ $rc -eq 0 ] || exit $rc
done
