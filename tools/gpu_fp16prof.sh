#!/bin/bash
# Kernel stats of the headline step in fp16 vs bf16 (same box): where the fp16 path loses time.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for D in fp16 bf16; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$D -o run --output-format csv -- python3 bench.py --dtype $D --steps 2 --warmup 1 --ga 2 --no-telemetry > gpurun_out/prof_$D.log 2>&1 || { tail -20 gpurun_out/prof_$D.log; exit 1; }
  tail -1 gpurun_out/prof_$D.log | cut -c1-200
done
