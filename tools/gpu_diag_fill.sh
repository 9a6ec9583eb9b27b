#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/diag/fill_sources.py mixtral-8x7b > gpurun_out/fill_sources_mixtral.log 2>&1; rc=$?
tail -30 gpurun_out/fill_sources_mixtral.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u tools/diag/fill_sources.py llama3-8b > gpurun_out/fill_sources_llama.log 2>&1; rc=$?
tail -30 gpurun_out/fill_sources_llama.log; exit $rc
