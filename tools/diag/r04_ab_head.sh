# A/B of this session's tree (HEAD) against the session's starting revision (ab_old/, built in-tree): alternating
# runs on one box of the headline and the Mixtral 2-layer bench
set -e
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out
for i in 1 2; do
  for tree in ab_old .; do
    (cd $tree && timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-telemetry > $O/ab_llama_$i_$(basename $(pwd)).json 2>/dev/null; cat $O/ab_llama_$i_$(basename $(pwd)).json | python3 -c "import json,sys; d=json.load(sys.stdin); print('llama', '$tree', d['value'])" >> $O/ab_head.txt)
  done
done
for i in 1 2 3; do
  for tree in ab_old .; do
    (cd $tree && timeout -k 10 400 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 --no-telemetry 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('mixtral', '$tree', d['value'])" >> $O/ab_head.txt)
  done
done
cat $O/ab_head.txt
