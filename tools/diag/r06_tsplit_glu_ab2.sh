# Round 6 (experiment, not kept): the tail split also on the fused SwiGLU-backward dX launch, banded reduce (DLGM_GEMM_TSPLIT_GLU=1 vs 0),
# after the MFMA GEMM tests; the Mixtral 2-layer bench alternating, twice each.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/tsab6
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_mfma_gpu.py \
  > gpurun_out/r06/tsab6/test.log 2>&1 || { tail -30 gpurun_out/r06/tsab6/test.log; exit 1; }
tail -1 gpurun_out/r06/tsab6/test.log
for i in 1 2; do
  for v in 1 0; do
    DLGM_GEMM_TSPLIT_GLU=$v timeout -k 10 300 python -u tools/diag/r06_mixtral_ab.py > gpurun_out/r06/tsab6/g$v-$i.json 2> gpurun_out/r06/tsab6/g$v-$i.err
    rc=$?; echo "glu=$v run$i rc=$rc $(python3 -c "import json; d=json.loads(open('gpurun_out/r06/tsab6/g$v-$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['extra']['mfu_vs_2.5PF_dense_bf16'])" 2>/dev/null)"
    [ $rc -eq 0 ] || exit $rc
  done
done
