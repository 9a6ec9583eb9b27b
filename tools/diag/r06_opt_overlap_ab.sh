# Round 6: Mixtral 2-layer bench, the overlapped optimizer (--optimizer-overlap on) vs the flat AdamW (default), alternating.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/ovab
for i in 1 2; do
  for v in base ovl; do
    VARIANT=$v timeout -k 10 300 python -u tools/diag/r06_mixtral_ab.py > gpurun_out/r06/ovab/$v$i.json 2> gpurun_out/r06/ovab/$v$i.err
    rc=$?; echo "$v$i rc=$rc $(python3 -c "import json; d=json.loads(open('gpurun_out/r06/ovab/$v$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['extra']['mfu_vs_2.5PF_dense_bf16'])" 2>/dev/null)"
    [ $rc -eq 0 ] || exit $rc
  done
done
