# round-4 records at HEAD: Mixtral-8x7B 2-layer micro-batch sweep (mbs 1/2/4 x GA 4) and GPT-2-small ZeRO-1
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
for mbs in 1 2 4; do
  timeout -k 10 500 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --mbs $mbs --ga 4 --steps 6 --warmup 2 --no-telemetry >> $O/mixtral_mbs_sweep_r04.jsonl 2>> $O/mixtral_mbs_sweep_r04.err
done
timeout -k 10 300 python bench.py --model gpt2-small --seq 1024 --mbs 8 --ga 4 --zero 1 --steps 20 --warmup 2 --no-telemetry > $O/bench_gpt2_small_r04b.json 2> $O/bench_gpt2_small_r04b.err
echo "== done"
