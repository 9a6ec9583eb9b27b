# Round 5 flake probe, stage 2: unit-level device-side snapshots of the first three Mixtral EP-4 engines right after
# the Mixtral async-shadow tests (where the round-4 mismatch showed); see tools/diag/flake/zz_units.py.
# ZZ_TAP selects the MoE-internal clones (fewer taps = less perturbation of the timing).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/digest
cat tools/diag/flake/zz_units.py >> tests/test_shadow_async_gpu.py
# the round-4 pre-state: every earlier engine of the file ran with the (then default) overlapped optimizer
if [ "${OVERLAP_PRE:-1}" = 1 ]; then
  sed -i 's/scheduler="constant", grad_clip=1.0)$/scheduler="constant", grad_clip=1.0, optimizer_overlap=True)/' tests/test_shadow_async_gpu.py
  grep -c 'grad_clip=1.0, optimizer_overlap=True)' tests/test_shadow_async_gpu.py
fi
K='swiglu or moe or mixtral or expert or mlp or zz_units'
D='tests/test_shadow_async_gpu.py::test_overlapped_optimizer_waits_per_group[mixtral-tiny-4-kw3]'
for tap in ${TAPS:-logits}; do
  ZZ_VAR=${tap#*:}; tap=${tap%%:*}; [ "$ZZ_VAR" = "$tap" ] && ZZ_VAR=""
  ZZ_VAR=$ZZ_VAR ZZ_TAP=$tap timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -s --timeout 250 --timeout-method thread \
      -p no:cacheprovider -k "$K" --deselect "$D" > gpurun_out/digest/units_$tap.txt 2>&1; rc=$?
  cp gpurun_out/digest/units_report.json gpurun_out/digest/units_report_${tap}${ZZ_VAR:+_$ZZ_VAR}.json
  echo "tap $tap rc=$rc: $(grep -E 'passed|failed' gpurun_out/digest/units_$tap.txt | tail -1)"
  case $rc in 0|1) ;; *) exit $rc;; esac
done
