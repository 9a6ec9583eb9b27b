set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "flash" > gpurun_out/pytest_attn.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_attn.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_attn.log | head -20; exit $rc; }
timeout -k 10 300 python tools/bench_kernels.py --only attn > gpurun_out/attn_bench.json 2> gpurun_out/attn_bench.err; rc=$?
cat gpurun_out/attn_bench.json; exit $rc
