#!/bin/bash
# Round 6 shadow-divergence reproducer runner (profiles/shadow_divergence_hunt_r06.json lists every run's settings):
#   bash tools/diag/r06_stress.sh TAG [VAR=value ...]
# runs tools/diag/r06_shadow_stress.py with those variables (REPS, LOOP_MODE=sync|async, CASES, DLGM_FORCE_REFERENCE,
# POISON, AUDIT, VARIANT, MESH_ALLOC, MESH_KEEP, AMD_SERIALIZE_KERNEL, ...) and prints the mismatch counts per case.
set -o pipefail
mkdir -p gpurun_out/r06/stress
export HSA_ENABLE_IPC_MODE_LEGACY=0
tag=${1:?tag}; shift
env "$@" timeout -k 10 300 python -u tools/diag/r06_shadow_stress.py > gpurun_out/r06/stress/$tag.log 2>&1
rc=$?
echo "$tag rc=$rc"; grep -E "async_mismatches" gpurun_out/r06/stress/$tag.log | grep -v '"env"' \
  | python3 -c "import sys,json; d={k: v['async_mismatches'] for l in sys.stdin for k, v in json.loads(l).items()}; print(sum(d.values()), d)"
! grep -q "HSA_STATUS_ERROR" gpurun_out/r06/stress/$tag.log && [ $rc -eq 0 ]
