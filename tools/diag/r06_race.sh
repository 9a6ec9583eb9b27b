# Round 6: the round-4 "first engine differs" mismatch under the poisoned-allocation and stream-audit debug modes,
# on the round-4 tree (_bisect/r04, warm-up removed from its test) and at HEAD; then the 1-GPU baseline bench.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06
K='overlapped_optimizer'
step() {  # name, dir, env, pytest args
  local name=$1 dir=$2 envs=$3; shift 3
  (cd $dir && env $envs timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread -p no:cacheprovider "$@" \
      > $GRAFT_REPO_ROOT/gpurun_out/r06/$name.log 2>&1); local rc=$?
  echo "$name rc=$rc: $(grep -E 'passed|failed|error' gpurun_out/r06/$name.log | tail -1)"
  case $rc in 0|1) return 0;; *) exit $rc;; esac
}
step audit_selftest_head . DLGM_STREAM_AUDIT=0 tests/test_stream_audit.py -m gpu
step poison_r04 _bisect/r04 DLGM_POISON_ALLOC=1 tests/test_shadow_async_gpu.py -m gpu -k "$K"
step poison_head . DLGM_POISON_ALLOC=1 tests/test_shadow_async_gpu.py -m gpu -k "$K"
step audit_r04 _bisect/r04 DLGM_STREAM_AUDIT=1 tests/test_shadow_async_gpu.py -m gpu -k "$K"
step audit_head . DLGM_STREAM_AUDIT=1 tests/test_shadow_async_gpu.py -m gpu
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/bench_base.json 2> gpurun_out/r06/bench_base.err
echo "bench rc=$?: $(cat gpurun_out/r06/bench_base.json)"
