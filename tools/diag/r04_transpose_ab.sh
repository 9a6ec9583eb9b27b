# transpose with one tile per wave (no grid-stride loop) vs ab_old/ (grid capped at 16 workgroups per CU):
# GEMM / transpose probe in both trees alternating (outputs carry sha digests), then the Mixtral 2-layer bench
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "transpose or dw_layout or wgrad" > $O/pytest_transpose.log 2>&1; rc=$?; fatal $rc pytest
echo "pytest: $(tail -1 $O/pytest_transpose.log)"
for r in 1 2; do
  for tree in ab_old .; do
    (cd $tree && ITERS=10 timeout -k 10 300 python tools/gemm_sched_ab.py 2>/dev/null | sed "s/^{/{\"tree\": \"$(basename $(pwd))\", /" >> $O/transpose_grid_ab.jsonl); rc=$?; fatal $rc probe
  done
done
for i in 1 2 3; do
  for tree in ab_old .; do
    (cd $tree && timeout -k 10 400 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 --no-telemetry 2>/dev/null > $O/tmx_${i}_$(basename $(pwd)).json); rc=$?; fatal $rc mixtral
  done
done
echo done
