# round-4 batch 8: LDS-staged bf16 and fp32 GEMM epilogues -- GEMM GPU tests, probe (bit-exactness vs the previous sha), Mixtral x2
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gemm_mfma_gpu.py tests/test_engine_numerics.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "gemm or grouped or mfma or mixtral or moe or expert or stats" > $O/pytest_b9.log 2>&1 || { tail -30 $O/pytest_b9.log; exit 1; }
tail -1 $O/pytest_b9.log
timeout -k 10 240 python tools/gemm_sched_ab.py >> $O/sched_ab9.jsonl
for i in 1 2; do
  timeout -k 10 400 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 --no-telemetry >> $O/mixtral_b9.jsonl 2>> $O/mixtral_b9.err
done
echo "== done"
