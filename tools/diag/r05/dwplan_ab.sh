# Round 5: dW operand-layout plan A/B on the headline config (alternating runs): the cost model's picks vs
# every dW forced to TN (both operands K-contiguous through the HIP transpose).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/digest
for r in 1 2; do
  for plan in auto TN; do
    DLGM_DW_PLAN=$plan timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-telemetry \
        > gpurun_out/digest/dwplan_${plan}_$r.log 2>&1 || exit $?
    echo "$plan run $r: $(grep '^{' gpurun_out/digest/dwplan_${plan}_$r.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"], d["ms_per_step"])')"
  done
done
