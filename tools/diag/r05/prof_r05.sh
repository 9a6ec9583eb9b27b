# Round 5 profiles at HEAD: (1) Mixtral-8x7B 2 layers, mbs 1 x GA 4, seq 4096: kernel TRACE (dispatch order, grid
# sizes) + stats; (2) the Llama-3-8B headline config: kernel stats. Bench lines go to the logs.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_mix_r05 gpurun_out/prof_head_r05
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mix_r05 -o run -- \
    python3 bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --mbs 1 --ga 4 --steps 3 --warmup 2 --no-telemetry \
    > gpurun_out/prof_mix_r05/bench.log 2>&1
rc=$?; echo "mix rc=$rc"; grep '^{' gpurun_out/prof_mix_r05/bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_head_r05 -o run -- \
    python3 bench.py --steps 3 --warmup 2 --no-telemetry > gpurun_out/prof_head_r05/bench.log 2>&1
rc=$?; echo "head rc=$rc"; grep '^{' gpurun_out/prof_head_r05/bench.log | cut -c1-300
find gpurun_out/prof_mix_r05 gpurun_out/prof_head_r05 -name "*kernel_trace.csv" -size +20M -delete
exit $rc
