set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python tools/tune_gemms.py --max-ms 10 --max-iters 10 2>&1 | grep -v amdgpu.ids | tee gpurun_out/tune.log
rc=$?
cp -r distributed_llm_training_gpu_manager_amd/tuned gpurun_out/ ; exit $rc
