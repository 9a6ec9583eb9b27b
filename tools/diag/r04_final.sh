# round-4 closing run: full GPU suite + smoke at HEAD, then HEAD vs the round's starting tree (ab_old/, built
# in-tree) alternating on one box: Mixtral 2-layer x3 each, headline x2 each
set -e
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu_final2.log 2>&1 || { tail -40 $O/pytest_gpu_final2.log; exit 1; }
tail -2 $O/pytest_gpu_final2.log
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke_final2.log 2>&1 || { tail -20 $O/smoke_final2.log; exit 1; }
tail -2 $O/smoke_final2.log
for i in 1 2 3; do
  for tree in ab_old .; do
    (cd $tree && timeout -k 10 400 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 --no-telemetry 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('mixtral', '$tree', d['value'])" >> $O/ab_final2.txt)
  done
done
for i in 1 2; do
  for tree in ab_old .; do
    (cd $tree && timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-telemetry 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('llama', '$tree', d['value'])" >> $O/ab_final2.txt)
  done
done
cat $O/ab_final2.txt
