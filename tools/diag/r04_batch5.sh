# round-4 batch 5: transpose probe, then the full round validation (GPU suite, smoke, kernel bench, headline bench,
# rocprof kernel stats) and a Mixtral 2-layer record with its kernel trace
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 240 python tools/gemm_sched_ab.py >> $O/sched_ab5.jsonl
echo "== probe done"
BENCH_STEPS=5 bash tools/gpu_round.sh all > $O/round_r4b.log 2>&1 || { tail -40 $O/round_r4b.log; exit 1; }
tail -3 $O/round_r4b.log
timeout -k 10 400 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 > $O/bench_mixtral_2l_r04c.json 2> $O/bench_mixtral_2l_r04c.err
cut -c1-300 $O/bench_mixtral_2l_r04c.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mixtral_r04c -o run -- python3 bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 2 --warmup 1 --no-telemetry --comm-sweep off --mesh-sweep off > $O/prof_mixtral_r04c.log 2>&1
echo "== all done"
