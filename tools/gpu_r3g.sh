#!/bin/bash
# w64 forward attention: numerics, then interleaved A/B against the default forward at the headline shape.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "w64 or dkdv_sp or fwd_bwd or headline or rescale or dq_from or fused_dqkv" -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_w64.log 2>&1; rc=$?
tail -12 gpurun_out/pytest_w64.log; [ $rc -eq 0 ] || exit $rc
DLGM_AB="w64:fwd:DLGM_ATTN_FWD=w64,sepdelta:bwd:DLGM_ATTN_DELTA_IN_DQ=0,sp:bwd:DLGM_ATTN_DKDV=sp" timeout -k 10 300 python tools/bench_kernels.py --only attn_ab > gpurun_out/attn_ab_w64.json 2> gpurun_out/attn_ab_w64.err; rc=$?
cat gpurun_out/attn_ab_w64.json; tail -3 gpurun_out/attn_ab_w64.err; exit $rc
