# MFMA GEMM / transpose probe (tools/gemm_sched_ab.py): timings, then PMC passes, one counter group per run
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_gemm
for sc in 0 1; do
  DLGM_GEMM_SCHED=$sc timeout -k 10 240 python tools/gemm_sched_ab.py >> gpurun_out/sched_ab2.jsonl
done
export ITERS=3
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_gemm/p1 -- python3 tools/gemm_sched_ab.py
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/pmc_gemm/p2 -- python3 tools/gemm_sched_ab.py
