# Round 6: the stream audit's GPU self-test, then the audit over the round-4 tree's failing test and HEAD's
# shadow-async suite.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06
step() {  # name, dir, env, pytest args
  local name=$1 dir=$2 envs=$3; shift 3
  (cd $dir && env $envs timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread -p no:cacheprovider "$@" \
      > $GRAFT_REPO_ROOT/gpurun_out/r06/$name.log 2>&1); local rc=$?
  echo "$name rc=$rc: $(grep -E 'passed|failed|error' gpurun_out/r06/$name.log | tail -1)"
  case $rc in 0|1) return 0;; *) exit $rc;; esac
}
step audit_selftest_head . DLGM_STREAM_AUDIT=0 tests/test_stream_audit.py -m gpu
step audit_r04 _bisect/r04 DLGM_STREAM_AUDIT=1 tests/test_shadow_async_gpu.py -m gpu -k "${K:-overlapped_optimizer}"
step audit_head . DLGM_STREAM_AUDIT=1 tests/test_shadow_async_gpu.py -m gpu
