# Round 5: the side-stream block-reuse test with the fix (must pass) and with the row plan's record_stream removed
# (negative control: expected to fail), then the 70B resume probe.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/digest
T=tests/test_engine_numerics.py::test_side_stream_inputs_survive_block_reuse_gpu
timeout -k 10 240 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider "$T" \
    "tests/test_engine_numerics.py::test_side_stream_work_is_waited_for_gpu" > gpurun_out/digest/reuse_fixed.txt 2>&1
rc=$?; echo "fixed rc=$rc: $(grep -E 'passed|failed' gpurun_out/digest/reuse_fixed.txt | tail -1)"
[ $rc -eq 0 ] || exit $rc
M=distributed_llm_training_gpu_manager_amd/models/mixtral.py
cp $M /tmp/mixtral_keep.py
sed -i '/src.record_stream(side)/d' $M
grep -c "src.record_stream" $M
timeout -k 10 240 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider "$T" \
    > gpurun_out/digest/reuse_negative.txt 2>&1
rc=$?; echo "negative control rc=$rc: $(grep -E 'passed|failed' gpurun_out/digest/reuse_negative.txt | tail -1)"
cp /tmp/mixtral_keep.py $M
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 900 python -u tools/diag/r05/resume_probe.py > gpurun_out/digest/resume_probe.txt 2>&1
rc=$?; echo "resume probe rc=$rc"; tail -5 gpurun_out/digest/resume_probe.txt; exit $rc
