cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/digest
SIZE=48 VRAM=96 timeout -k 10 300 python -u tools/diag/r05/prefault_bench.py > gpurun_out/digest/prefault.txt 2>&1
rc=$?; echo "prefault rc=$rc"; tail -2 gpurun_out/digest/prefault.txt; [ $rc -eq 0 ] || exit $rc
T=tests/test_engine_numerics.py::test_side_stream_inputs_survive_block_reuse_gpu
timeout -k 10 240 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider "$T" \
    > gpurun_out/digest/reuse_fixed2.txt 2>&1
rc=$?; echo "fixed rc=$rc: $(grep -E 'passed|failed' gpurun_out/digest/reuse_fixed2.txt | tail -1)"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_runtime.py -k "shm" > gpurun_out/digest/shm_tests.txt 2>&1
rc=$?; echo "shm tests rc=$rc: $(grep -E 'passed|failed' gpurun_out/digest/shm_tests.txt | tail -1)"
[ $rc -eq 0 ] || exit $rc
M=distributed_llm_training_gpu_manager_amd/models/mixtral.py
cp $M /tmp/mixtral_keep.py
sed -i '/src.record_stream(side)/d' $M
grep -c "src.record_stream" $M
timeout -k 10 240 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider "$T" \
    > gpurun_out/digest/reuse_negative2.txt 2>&1
rc=$?; echo "negative control rc=$rc: $(grep -E 'passed|failed' gpurun_out/digest/reuse_negative2.txt | tail -1)"
grep -E "AssertionError|assert" gpurun_out/digest/reuse_negative2.txt | head -5
cp /tmp/mixtral_keep.py $M
case $rc in 0|1) exit 0;; *) exit $rc;; esac
