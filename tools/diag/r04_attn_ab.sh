# dK/dV staged fp32 partials (.) vs HEAD without it (ab_old/), alternating kernel benches on one box
set -e
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out
for i in 1 2 3; do
  for tree in ab_old .; do
    (cd $tree && timeout -k 10 300 python tools/bench_kernels.py 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('$tree', d['ab_bwd']['median_ms'], d['ab_fwd']['median_ms'])" >> $O/attn_ab.txt)
  done
done
cat $O/attn_ab.txt
