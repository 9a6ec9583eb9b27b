#!/bin/bash
# attention numerics with the in-tree build, then a same-device A/B of attention kernel builds
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attn or attention or flash" --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 &&
timeout -k 10 600 bash tools/ab_kernels.sh attn "$@" > gpurun_out/attn_ab.log 2>&1
