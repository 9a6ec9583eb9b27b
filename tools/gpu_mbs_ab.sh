#!/bin/bash
# Headline config at the same tokens per step: micro-batch 1 x GA 8 vs micro-batch 2 x GA 4 (one MI355X)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --mbs 1 --ga 8 --comm-sweep off > gpurun_out/mbs1_ga8.json 2> gpurun_out/mbs1_ga8.err &&
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 --mbs 2 --ga 4 --comm-sweep off > gpurun_out/mbs2_ga4.json 2> gpurun_out/mbs2_ga4.err
