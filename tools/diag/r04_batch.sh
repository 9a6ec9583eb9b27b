# round-4 batch: MFMA GEMM schedule / transpose probe, overlap + transpose GPU tests, optimizer-overlap A/B on the
# headline and Mixtral 2-layer benches, then PMC passes over the GEMM probe. Each step has its own time limit.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_gemm
O=gpurun_out
for sc in 0 1; do
  DLGM_GEMM_SCHED=$sc timeout -k 10 240 python tools/gemm_sched_ab.py >> $O/sched_ab2.jsonl
done
echo "== probe done"
timeout -k 10 400 python -u -m pytest tests/test_engine_numerics.py tests/test_kernels_gpu.py tests/test_gemm_mfma_gpu.py tests/test_moe_dw_layout.py -m gpu -x -q --timeout 120 --timeout-method thread -k "overlap or transpose or mfma or grouped or gemm or layout" > $O/pytest_overlap.log 2>&1 || { tail -30 $O/pytest_overlap.log; exit 1; }
tail -2 $O/pytest_overlap.log
timeout -k 10 600 python -u -m pytest tests/test_shadow_async_gpu.py tests/test_gpu_runtime.py tests/test_fp16_path.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_overlap2.log 2>&1 || { tail -30 $O/pytest_overlap2.log; exit 1; }
tail -2 $O/pytest_overlap2.log
for ov in on off on off; do
  timeout -k 10 400 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 --optimizer-overlap $ov --no-telemetry >> $O/mixtral_overlap_ab.jsonl 2>> $O/mixtral_overlap_ab.err
done
echo "== mixtral done"
for ov in on off; do
  timeout -k 10 600 python bench.py --steps 3 --warmup 1 --optimizer-overlap $ov --no-telemetry >> $O/llama_overlap_ab.jsonl 2>> $O/llama_overlap_ab.err
done
echo "== llama done"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export ITERS=3
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_gemm/p1 -- python3 tools/gemm_sched_ab.py > /dev/null
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS --output-format csv -d $O/pmc_gemm/p2 -- python3 tools/gemm_sched_ab.py > /dev/null
echo "== pmc done"
