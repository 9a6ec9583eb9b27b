set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python tools/tune_gemms.py > gpurun_out/tune.log 2>&1; rc=$?
grep -v "^{" gpurun_out/tune.log | tail -24; [ $rc -eq 0 ] || exit $rc
cp -r distributed_llm_training_gpu_manager_amd/tuned gpurun_out/ 
