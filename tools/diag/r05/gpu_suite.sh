# Round 5: the whole GPU suite at HEAD (as the driver runs it), then the fp16 headline config once with the timed
# fp16 hipBLASLt picks written to gpurun_out/tune (committed as tuned/gemm_lt_f16_v<ver>.json).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tune
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu_r05.log 2>&1
rc=$?; echo "suite rc=$rc: $(grep -E 'passed|failed' gpurun_out/pytest_gpu_r05.log | tail -1)"; [ $rc -eq 0 ] || exit $rc
DLGM_TUNE_CACHE=gpurun_out/tune timeout -k 10 200 python -u bench.py --dtype fp16 --steps 2 --warmup 1 --no-telemetry \
    > gpurun_out/bench_fp16_r05.log 2>&1
rc=$?; echo "fp16 rc=$rc: $(grep '^{' gpurun_out/bench_fp16_r05.log | cut -c1-160)"; ls gpurun_out/tune; exit $rc
