cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/tune_gemms.py --max-ms 10 --max-iters 10 > gpurun_out/tune.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/tune.log | tail -20
cp -r distributed_llm_training_gpu_manager_amd/tuned gpurun_out/ ; exit $rc
