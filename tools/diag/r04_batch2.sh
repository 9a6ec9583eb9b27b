# round-4 batch 2: GEMM schedule + transpose probe (incl. the engine's mode-2 dW), transpose/layout GPU tests,
# Mixtral 2-layer A/B of the side-stream W^T rebuild / dW re-layout (optimizer overlap off in both arms)
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
for sc in 0 1; do
  DLGM_GEMM_SCHED=$sc timeout -k 10 240 python tools/gemm_sched_ab.py >> $O/sched_ab3.jsonl
done
echo "== probe done"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_moe_dw_layout.py tests/test_engine_numerics.py -m gpu -x -q --timeout 120 --timeout-method thread -k "transpose or layout or mixtral or transposed or overlap" > $O/pytest_b2.log 2>&1 || { tail -30 $O/pytest_b2.log; exit 1; }
tail -2 $O/pytest_b2.log
for ss in 1 0 1 0 1 0; do
  DLGM_SIDE_STREAMS=$ss timeout -k 10 400 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 --optimizer-overlap off --no-telemetry >> $O/mixtral_side_ab.jsonl 2>> $O/mixtral_side_ab.err
done
echo "== mixtral done"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_overlap -- python3 bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 2 --warmup 1 --optimizer-overlap on --no-telemetry --comm-sweep off --mesh-sweep off > $O/prof_overlap.log 2>&1
echo "== trace done"
