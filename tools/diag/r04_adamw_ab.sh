# AdamW one-vector-per-lane grid + grad_stats 8-deep NT loads: optimizer GPU tests, kernel micro-bench in both
# trees, then HEAD vs the previous commit (ab_old/, built in-tree) alternating on one box
set -e
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "adam or optim or stats or scaler or overlap or engine" > $O/pytest_gpu_adamw.log 2>&1 || { tail -40 $O/pytest_gpu_adamw.log; exit 1; }
tail -2 $O/pytest_gpu_adamw.log
for tree in ab_old .; do
  (cd $tree && timeout -k 10 120 python tools/bench_kernels.py --only adamw > $O/bk_adamw_$(basename $(pwd)).json 2>/dev/null)
done
for i in 1 2 3; do
  for tree in ab_old .; do
    (cd $tree && timeout -k 10 400 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 --no-telemetry 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('mixtral', '$tree', d['value'])" >> $O/ab_adamw.txt)
  done
done
for i in 1 2; do
  for tree in ab_old .; do
    (cd $tree && timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-telemetry 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('llama', '$tree', d['value'])" >> $O/ab_adamw.txt)
  done
done
cat $O/ab_adamw.txt
