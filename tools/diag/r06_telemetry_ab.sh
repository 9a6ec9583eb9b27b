# Round 6: headline bench with the in-run amdsmi telemetry sampler (default, every 2 s) vs --no-telemetry, alternating.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/telab
for i in 1 2; do
  for v in tel notel; do
    extra=""; [ $v = notel ] && extra="--no-telemetry"
    timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 $extra > gpurun_out/r06/telab/$v$i.json 2> gpurun_out/r06/telab/$v$i.err
    rc=$?; echo "$v$i rc=$rc $(python3 -c "import json; d=json.loads(open('gpurun_out/r06/telab/$v$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
    [ $rc -eq 0 ] || exit $rc
  done
done
