# Round 6: stream-audit self-test (with a dump on failure), then HEAD's shadow-async + runtime suites under the audit.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06
step() {  # name, env, pytest args
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 400 python -u -m pytest -x -v --timeout 250 --timeout-method thread -p no:cacheprovider "$@" \
      > gpurun_out/r06/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc: $(grep -E 'passed|failed|error' gpurun_out/r06/$name.log | tail -1)"
  case $rc in 0|1) return 0;; *) exit $rc;; esac
}
step audit_selftest DLGM_STREAM_AUDIT=0 tests/test_stream_audit.py -m gpu
step audit_shadow DLGM_STREAM_AUDIT=1 tests/test_shadow_async_gpu.py -m gpu
step gpu_runtime DLGM_STREAM_AUDIT=0 tests/test_gpu_runtime.py -m gpu -k "shm_save"
