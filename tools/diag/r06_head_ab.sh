#!/bin/bash
# Round 6: same-box A/B of the headline bench, HEAD vs b0c3eeb (the commit of profiles/bench_r06_final.json; a git
# worktree under _ab/ with HEAD's native libraries), alternating, twice each.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/headab
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2; do
  for v in head old; do
    dir=.; [ $v = old ] && dir=_ab/b0c3eeb
    (cd $dir && timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5) \
      > gpurun_out/r06/headab/$v$i.json 2> gpurun_out/r06/headab/$v$i.err
    rc=$?; echo "$v$i rc=$rc $(python3 -c "import json; d=json.loads(open('gpurun_out/r06/headab/$v$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['extra']['telemetry']['power_w']['mean'])" 2>/dev/null)"
    [ $rc -eq 0 ] || exit $rc
  done
done
