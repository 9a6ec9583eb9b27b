# late round-4 batch: (1) the order-dependent Mixtral EP-4 mismatch with the caching allocator off, (2) the full GPU
# suite in default order at HEAD, (3) swiglu one-vector-per-lane micro-bench + Mixtral / Llama A/B vs ab_old/.
# A step that times out or crashes (124 / 134 / 137 / 139) ends the script; a plain test failure does not.
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
PYTORCH_NO_HIP_MEMORY_CACHING=1 PYTORCH_NO_CUDA_MEMORY_CACHING=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "swiglu or moe or mixtral or expert or mlp" > $O/flake_nocache.txt 2>&1; rc=$?; fatal $rc nocache
echo "nocache: $(grep -E 'passed|failed' $O/flake_nocache.txt | tail -1)"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu_late.log 2>&1; rc=$?; fatal $rc suite
echo "suite: $(tail -1 $O/pytest_gpu_late.log)"
for r in 1 2; do
  for tree in ab_old .; do
    (cd $tree && timeout -k 10 120 python tools/bench_kernels.py --only swiglu > $O/bk_swiglu_${r}_$(basename $(pwd)).json 2>/dev/null); rc=$?; fatal $rc bk
  done
done
for i in 1 2 3; do
  for tree in ab_old .; do
    (cd $tree && timeout -k 10 400 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 --no-telemetry 2>/dev/null > $O/mx_${i}_$(basename $(pwd)).json); rc=$?; fatal $rc mixtral
  done
done
for i in 1 2; do
  for tree in ab_old .; do
    (cd $tree && timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-telemetry 2>/dev/null > $O/ll_${i}_$(basename $(pwd)).json); rc=$?; fatal $rc llama
  done
done
echo done
