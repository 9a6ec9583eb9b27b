# Round 5: locate the first op whose output differs between the first and second Mixtral EP-4 engine after the
# selection that precedes the round-4 overlapped-optimizer mismatch. The probe is appended to
# tests/test_shadow_async_gpu.py (on the box only) so it runs exactly where the mismatching test ran.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/digest
sed -n '/^SKIP = /,$p' tools/diag/flake/test_zz_digest.py | sed 's/_engine_run/_zz_engine_run/g' > /tmp/zz_body.py
{ echo "import hashlib, json, os"; echo "from torch.utils._python_dispatch import TorchDispatchMode"; echo "from torch.utils._pytree import tree_leaves"; cat /tmp/zz_body.py; } >> tests/test_shadow_async_gpu.py
K='swiglu or moe or mixtral or expert or mlp or zz_digest'
D='tests/test_shadow_async_gpu.py::test_overlapped_optimizer_waits_per_group[mixtral-tiny-4-kw3]'
for dg in 0 1; do
  DIGEST=$dg timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -s --timeout 400 --timeout-method thread \
    -p no:cacheprovider -k "$K" --deselect "$D" > gpurun_out/digest/run_$dg.txt 2>&1; rc=$?
  echo "digest=$dg rc=$rc: $(grep -E 'passed|failed' gpurun_out/digest/run_$dg.txt | tail -1)"
  grep -E '^\{"n_ops' gpurun_out/digest/run_$dg.txt
  case $rc in 0|1) ;; *) exit $rc;; esac
done
