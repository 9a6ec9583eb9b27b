#!/bin/bash
# Round 6: the LM head's dW once per step (default) vs per micro-batch (VARIANT=nohead): the GPU suite first, then the
# Mixtral 2-layer bench alternating, twice each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/hdab
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r06/hdab/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc: $(tail -1 gpurun_out/r06/hdab/pytest_gpu.log)"
grep -E "^FAILED|^ERROR" gpurun_out/r06/hdab/pytest_gpu.log | head -20
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in base nohead; do
    VARIANT=$v timeout -k 10 300 python -u tools/diag/r06_mixtral_ab.py > gpurun_out/r06/hdab/$v$i.json 2> gpurun_out/r06/hdab/$v$i.err
    rc=$?; echo "$v$i rc=$rc $(python3 -c "import json; d=json.loads(open('gpurun_out/r06/hdab/$v$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['extra']['mfu_vs_2.5PF_dense_bf16'])" 2>/dev/null)"
    [ $rc -eq 0 ] || exit $rc
  done
done
