# rmsnorm forward holding the row as 16-bit values: bit-identity digests and micro-bench in both trees
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "rmsnorm or norm" > $O/pytest_rmsnorm.log 2>&1; rc=$?; fatal $rc pytest
echo "pytest: $(tail -1 $O/pytest_rmsnorm.log)"
for tree in ab_old .; do
  (cd $tree && timeout -k 10 120 python $GRAFT_REPO_ROOT/tools/diag/rmsnorm_digest.py 2>/dev/null | sed "s/^{/{\"tree\": \"$(basename $(pwd))\", /"); rc=$?; fatal $rc digest
done
for r in 1 2 3; do
  for tree in ab_old .; do
    (cd $tree && timeout -k 10 120 python tools/bench_kernels.py --only rmsnorm 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('$tree', d['add_rmsnorm_fwd'], d['rmsnorm_bwd'])"); rc=$?; fatal $rc bk
  done
done
