# Round 5: the headline on one box, HEAD vs the round-4 tree (3208a31, built in _ab/r04), alternating, plus the
# dW cost probe at HEAD (T vs 2T along K, per layout).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-telemetry > gpurun_out/ab/head_$r.log 2>&1 || exit $?
  echo "head run $r: $(grep '^{' gpurun_out/ab/head_$r.log | cut -c60-140)"
  (cd _ab/r04 && timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-telemetry > ../../gpurun_out/ab/r04_$r.log 2>&1) || exit $?
  echo "r04 run $r: $(grep '^{' gpurun_out/ab/r04_$r.log | cut -c60-140)"
done
timeout -k 10 300 python -u tools/probe_dw_cost.py --out gpurun_out/ab/probe_dw_cost_r05.json > gpurun_out/ab/probe_dw.log 2>&1
echo "probe rc=$?"
