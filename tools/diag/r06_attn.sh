# Round 6: stored-dS attention backward -- numerics (bf16 / fp16, every shape class), interleaved A/B against the
# two-recompute backward at the headline shape, then the suites the previous audit run flagged.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06
step() {  # name, env, cmd...
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 400 "$@" > gpurun_out/r06/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc: $(grep -E 'passed|failed|error|ab_' gpurun_out/r06/$name.log | tail -3 | tr '\n' ' ')"
  case $rc in 0|1) return 0;; *) exit $rc;; esac
}
step attn_tests X=1 python -u -m pytest -x -v --timeout 250 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_kernels_gpu.py tests/test_kernels_fp16_gpu.py -k "flash or attention"
step attn_ab DLGM_AB=rec:bwd:DLGM_ATTN_BWD=recompute python -u tools/bench_kernels.py --only attn_ab
step audit_fixes DLGM_STREAM_AUDIT=1 python -u -m pytest -v --timeout 250 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_mesh_engine_gpu.py tests/test_xgmi_mesh_gpu.py tests/test_shadow_async_gpu.py
