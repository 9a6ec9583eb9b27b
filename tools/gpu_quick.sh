#!/bin/bash
# Quick GPU check of a subset of tests: tools/gpu_quick.sh <pytest args...>
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" > gpurun_out/pytest_quick.log 2>&1; rc=$?
tail -25 gpurun_out/pytest_quick.log
exit $rc
