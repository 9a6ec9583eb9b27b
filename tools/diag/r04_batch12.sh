# transpose rows padded to 128-B lines: GPU tests (layout, MoE, engine), probe, Mixtral x2
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_moe_dw_layout.py tests/test_gemm_mfma_gpu.py tests/test_kernels_gpu.py tests/test_engine_numerics.py tests/test_xgmi_mesh_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "transpose or layout or moe or mixtral or expert or grouped or gemm or mfma" > $O/pytest_b14.log 2>&1 || { tail -30 $O/pytest_b14.log; exit 1; }
tail -1 $O/pytest_b14.log
timeout -k 10 300 python tools/gemm_sched_ab.py > $O/sched_ab14.jsonl
for i in 1 2; do
  timeout -k 10 400 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 --no-telemetry >> $O/mixtral_b14.jsonl 2>> $O/mixtral_b14.err
done
echo "== done"
