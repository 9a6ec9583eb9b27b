df -h /tmp $GRAFT_REPO_ROOT /dev/shm 2>&1 | tail -4
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/prof_bench.sh
