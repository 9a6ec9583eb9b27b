set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k rmsnorm --timeout 120 --timeout-method thread > gpurun_out/pytest_rms.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_rms.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_kernels.py --only rmsnorm > gpurun_out/bench_rms.json 2>/dev/null; cat gpurun_out/bench_rms.json
