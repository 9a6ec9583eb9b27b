#!/bin/bash
# fp16 headline step kernel stats (where the fp16 path loses against bf16).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fp16 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --ga 2 --dtype fp16 > gpurun_out/prof_fp16.log 2>&1; rc=$?
tail -2 gpurun_out/prof_fp16.log; find gpurun_out/prof_fp16 -name "*kernel_stats*"; exit $rc
