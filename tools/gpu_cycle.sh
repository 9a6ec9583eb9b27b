# One GPU measurement cycle: gpu tests -> 1-GPU bench -> rocprofv3 kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
cat gpurun_out/bench.json; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench.err; exit $rc; }
timeout -k 10 600 bash tools/prof_bench.sh
