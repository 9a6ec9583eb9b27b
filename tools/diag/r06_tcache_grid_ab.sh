# Round 6 (experiment, knob since removed): the side-stream W^T rebuild with its transposes' grid capped (DLGM_TCACHE_BLOCKS=128 / 64) vs the
# kernel's own grid (0), Mixtral 2-layer bench, alternating.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/tgab
for i in 1 2; do
  for v in 0 128 64; do
    DLGM_TCACHE_BLOCKS=$v timeout -k 10 300 python -u tools/diag/r06_mixtral_ab.py > gpurun_out/r06/tgab/b$v-$i.json 2> gpurun_out/r06/tgab/b$v-$i.err
    rc=$?; echo "blocks=$v run$i rc=$rc $(python3 -c "import json; d=json.loads(open('gpurun_out/r06/tgab/b$v-$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['extra']['mfu_vs_2.5PF_dense_bf16'])" 2>/dev/null)"
    [ $rc -eq 0 ] || exit $rc
  done
done
