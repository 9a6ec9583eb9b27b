cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/digest
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_runtime.py -k "shm" > gpurun_out/digest/shm_tests2.txt 2>&1
rc=$?; echo "shm tests rc=$rc: $(grep -E 'passed|failed' gpurun_out/digest/shm_tests2.txt | tail -1)"; [ $rc -eq 0 ] || exit $rc
DRILLS=spot TAG=r05_spot3 timeout -k 10 600 bash tools/gpu_drills_mixtral.sh > gpurun_out/drillmix_spot3.txt 2>&1
rc=$?; echo "spot rc=$rc"; exit $rc
