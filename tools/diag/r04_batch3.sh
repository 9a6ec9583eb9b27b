# round-4 batch 3: MFMA GEMM (per-mode DMA placement) + MoE GPU tests, optimizer-overlap A/B with the
# per-group wait at the point of use (Mixtral 2-layer x3, Llama-3-8B x2), kernel trace of the overlapped step
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gemm_mfma_gpu.py tests/test_moe_dw_layout.py tests/test_engine_numerics.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm or grouped or mfma or layout or mixtral or overlap or transpose or moe" > $O/pytest_b3.log 2>&1 || { tail -30 $O/pytest_b3.log; exit 1; }
tail -2 $O/pytest_b3.log
timeout -k 10 240 python tools/gemm_sched_ab.py >> $O/sched_ab4.jsonl
for ov in on off on off on off; do
  timeout -k 10 400 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 --optimizer-overlap $ov --no-telemetry >> $O/mixtral_overlap_ab2.jsonl 2>> $O/mixtral_overlap_ab2.err
done
echo "== mixtral done"
for ov in on off; do
  timeout -k 10 600 python bench.py --steps 3 --warmup 1 --optimizer-overlap $ov --no-telemetry >> $O/llama_overlap_ab2.jsonl 2>> $O/llama_overlap_ab2.err
done
echo "== llama done"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_overlap2 -- python3 bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 2 --warmup 1 --optimizer-overlap on --no-telemetry --comm-sweep off --mesh-sweep off > $O/prof_overlap2.log 2>&1
echo "== trace done"
