# Round 6: tail_reduce_kernel with 8 row-band blocks per tile (DLGM_GEMM_TRED_BANDS=8, default) vs one block per tile
# (=1), after the MFMA GEMM tests; the Mixtral 2-layer bench alternating, twice each.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/trab
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_mfma_gpu.py \
  > gpurun_out/r06/trab/test.log 2>&1 || { tail -30 gpurun_out/r06/trab/test.log; exit 1; }
tail -1 gpurun_out/r06/trab/test.log
for i in 1 2; do
  for v in 8 1; do
    DLGM_GEMM_TRED_BANDS=$v timeout -k 10 300 python -u tools/diag/r06_mixtral_ab.py > gpurun_out/r06/trab/b$v-$i.json 2> gpurun_out/r06/trab/b$v-$i.err
    rc=$?; echo "bands=$v run$i rc=$rc $(python3 -c "import json; d=json.loads(open('gpurun_out/r06/trab/b$v-$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['extra']['mfu_vs_2.5PF_dense_bf16'])" 2>/dev/null)"
    [ $rc -eq 0 ] || exit $rc
  done
done
