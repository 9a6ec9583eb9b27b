set -e
mkdir -p gpurun_out
for sc in 0 1 2 0 1 2; do
  DLGM_GEMM_SCHED=$sc timeout -k 10 240 python tools/gemm_sched_ab.py >> gpurun_out/sched_ab.jsonl
done
