# Round 6: grouped-M tail split -- the MFMA GEMM tests, then the Mixtral 2-layer bench with DLGM_GEMM_TSPLIT=1 (tail
# split, every grouped-M bf16 launch with K >= 4096) / 0 (the round-4 split-K rule), alternating, twice each.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/tsab2
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_mfma_gpu.py \
  > gpurun_out/r06/tsab2/test.log 2>&1 || { tail -30 gpurun_out/r06/tsab2/test.log; exit 1; }
tail -3 gpurun_out/r06/tsab2/test.log
for i in 1 2; do
  for v in 1 0; do
    DLGM_GEMM_TSPLIT=$v timeout -k 10 300 python -u tools/diag/r06_mixtral_ab.py > gpurun_out/r06/tsab2/f$v-$i.json 2> gpurun_out/r06/tsab2/f$v-$i.err
    rc=$?; echo "tsplit=$v run$i rc=$rc $(python3 -c "import json; d=json.loads(open('gpurun_out/r06/tsab2/f$v-$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['extra']['mfu_vs_2.5PF_dense_bf16'])" 2>/dev/null)"
    [ $rc -eq 0 ] || exit $rc
  done
done
