#!/bin/bash
# Non-headline model records on one MI355X: Mixtral-8x7B at 2 layers (eager and HIP-graph captured), GPT-2-small
# ZeRO-1 (BASELINE config 1's model). Each run has its own time limit; a failure ends the session.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TAG:-r04}
timeout -k 10 400 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 \
    > gpurun_out/bench_mixtral_2l_$T.json 2> gpurun_out/bench_mixtral_2l_$T.err || { tail -20 gpurun_out/bench_mixtral_2l_$T.err; exit 1; }
cut -c1-400 gpurun_out/bench_mixtral_2l_$T.json
timeout -k 10 400 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 --hip-graphs \
    > gpurun_out/bench_mixtral_2l_graph_$T.json 2> gpurun_out/bench_mixtral_2l_graph_$T.err || { tail -20 gpurun_out/bench_mixtral_2l_graph_$T.err; exit 1; }
cut -c1-400 gpurun_out/bench_mixtral_2l_graph_$T.json
timeout -k 10 300 python bench.py --model gpt2-small --seq 1024 --mbs 8 --ga 4 --zero 1 --steps 20 --warmup 2 \
    > gpurun_out/bench_gpt2_small_$T.json 2> gpurun_out/bench_gpt2_small_$T.err || { tail -20 gpurun_out/bench_gpt2_small_$T.err; exit 1; }
cut -c1-400 gpurun_out/bench_gpt2_small_$T.json
