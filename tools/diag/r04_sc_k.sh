set -e
cd "$GRAFT_REPO_ROOT"
for t in 0 1 0 1; do
  if [ $t = 1 ]; then export DLGM_TMP_SC=1; else unset DLGM_TMP_SC; fi
  timeout -k 10 300 python tools/gemm_sched_ab.py >> gpurun_out/sc_k.jsonl
done
