# Round 6 (experiment, not kept): the deferred expert dW flush's operand re-layout started beside the last micro-batch's dX GEMMs
# Round 6: the deferred expert dW flush's operand re-layout started beside the last micro-batch's dX GEMMs
# (DLGM_MOE_EARLY_FLUSH=1, default) vs after them (=0): engine / MoE GPU tests first, then the Mixtral 2-layer bench
# alternating, twice each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/efab
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_engine_numerics.py tests/test_gemm_mfma_gpu.py tests/test_shadow_async_gpu.py > gpurun_out/r06/efab/test.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/r06/efab/test.log)"; grep -E "^FAILED|^ERROR" gpurun_out/r06/efab/test.log | head
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in 1 0; do
    DLGM_MOE_EARLY_FLUSH=$v timeout -k 10 300 python -u tools/diag/r06_mixtral_ab.py > gpurun_out/r06/efab/e$v-$i.json 2> gpurun_out/r06/efab/e$v-$i.err
    rc=$?; echo "early=$v run$i rc=$rc $(python3 -c "import json; d=json.loads(open('gpurun_out/r06/efab/e$v-$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['extra']['mfu_vs_2.5PF_dense_bf16'])" 2>/dev/null)"
    [ $rc -eq 0 ] || exit $rc
  done
done
