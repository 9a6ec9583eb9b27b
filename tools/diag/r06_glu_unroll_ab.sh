# Round 6 (experiment, not kept): the fused SwiGLU-backward epilogue's row loop unrolled 8x (more gate / up loads in flight; a worktree
# build under _ab/unroll8) vs 2x (HEAD): Mixtral 2-layer bench alternating, twice each.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/u8ab2
for i in 1 2; do
  for v in head u8; do
    dir=.; [ $v = u8 ] && dir=_ab/unroll8
    (cd $dir && timeout -k 10 300 python -u tools/diag/r06_mixtral_ab.py) > gpurun_out/r06/u8ab2/$v$i.json 2> gpurun_out/r06/u8ab2/$v$i.err
    rc=$?; echo "$v$i rc=$rc $(python3 -c "import json; d=json.loads(open('gpurun_out/r06/u8ab2/$v$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['extra']['mfu_vs_2.5PF_dense_bf16'])" 2>/dev/null)"
    [ $rc -eq 0 ] || exit $rc
  done
done
