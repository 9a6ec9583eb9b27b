#!/bin/bash
# Round-3 closing records: Mixtral 2-layer micro-batch sweep on the final MoE path, GPT-2-small, headline 10 steps.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for MBS in 2 4 8; do
  timeout -k 10 400 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --mbs $MBS --ga 4 --steps 4 --warmup 2 --no-telemetry > gpurun_out/bench_mixtral_mbs$MBS.json 2> gpurun_out/bench_mixtral_mbs$MBS.err || { tail -10 gpurun_out/bench_mixtral_mbs$MBS.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_mixtral_mbs$MBS.json'));print('mixtral mbs $MBS', d['value'],d['ms_per_step'],d['extra']['mfu_vs_2.5PF_dense_bf16'],d['extra']['peak_GiB_max_over_ranks'])"
done
timeout -k 10 300 python bench.py --model gpt2-small --seq 1024 --mbs 8 --ga 4 --zero 1 --steps 20 --warmup 2 --no-telemetry > gpurun_out/bench_gpt2.json 2> gpurun_out/bench_gpt2.err || { tail -10 gpurun_out/bench_gpt2.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_gpt2.json'));print('gpt2', d['value'],d['ms_per_step'])"
timeout -k 10 900 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_headline10.json 2> gpurun_out/bench_headline10.err || { tail -10 gpurun_out/bench_headline10.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_headline10.json'));print('headline', d['value'],d['ms_per_step'],d['extra']['mfu_vs_2.5PF_dense_bf16'])"
