# round-4 batch 6: MoE permute in registers -- MoE / mesh EP GPU tests, Mixtral 2-layer bench x2, kernel trace
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_numerics.py tests/test_xgmi_mesh_gpu.py tests/test_gemm_mfma_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "moe or mixtral or permute or expert or grouped" > $O/pytest_b6.log 2>&1 || { tail -30 $O/pytest_b6.log; exit 1; }
tail -1 $O/pytest_b6.log
for i in 1 2; do
  timeout -k 10 400 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 --no-telemetry >> $O/mixtral_b6.jsonl 2>> $O/mixtral_b6.err
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b6 -o run -- python3 bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 2 --warmup 1 --no-telemetry --comm-sweep off --mesh-sweep off > $O/prof_b6.log 2>&1
echo "== done"
