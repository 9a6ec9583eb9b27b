set -e
cd "$GRAFT_REPO_ROOT"
for t in 0 1 0 1; do
  if [ $t = 1 ]; then export DLGM_TMP_SPLIT=1; else unset DLGM_TMP_SPLIT; fi
  timeout -k 10 300 python tools/gemm_sched_ab.py >> gpurun_out/split.jsonl
done
for t in 0 1 0 1; do
  if [ $t = 1 ]; then export DLGM_TMP_SPLIT=1; else unset DLGM_TMP_SPLIT; fi
  timeout -k 10 400 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 --no-telemetry >> gpurun_out/split_mix.jsonl 2>/dev/null
done
