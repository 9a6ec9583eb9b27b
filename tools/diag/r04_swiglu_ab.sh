# swiglu one vector per lane (no grid-stride loop, no per-lane 64-bit division): swiglu / MoE GPU tests, kernel
# micro-bench in both trees, then HEAD vs the previous commit (ab_old/, built in-tree) alternating on one box
set -e
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "swiglu or moe or mixtral or expert or mlp" > $O/pytest_gpu_swiglu.log 2>&1 || { tail -40 $O/pytest_gpu_swiglu.log; exit 1; }
tail -2 $O/pytest_gpu_swiglu.log
for r in 1 2; do
  for tree in ab_old .; do
    (cd $tree && timeout -k 10 120 python tools/bench_kernels.py --only swiglu > $O/bk_swiglu_${r}_$(basename $(pwd)).json 2>/dev/null)
  done
done
for i in 1 2 3; do
  for tree in ab_old .; do
    (cd $tree && timeout -k 10 400 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 --no-telemetry 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('mixtral', '$tree', d['value'], d.get('mfu'))" >> $O/ab_swiglu.txt)
  done
done
for i in 1 2; do
  for tree in ab_old .; do
    (cd $tree && timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-telemetry 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('llama', '$tree', d['value'])" >> $O/ab_swiglu.txt)
  done
done
cat $O/ab_swiglu.txt
