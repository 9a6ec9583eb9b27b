# Round 6: the whole GPU suite under the stream-ordering audit (DLGM_STREAM_AUDIT=1), every failure listed.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06
DLGM_STREAM_AUDIT=1 timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r06/pytest_gpu_audit3.log 2>&1; rc=$?
echo "rc=$rc: $(grep -E 'passed|failed' gpurun_out/r06/pytest_gpu_audit3.log | tail -1)"
grep -E "FAILED|ERROR" gpurun_out/r06/pytest_gpu_audit3.log | head -40
case $rc in 0|1) exit 0;; *) exit $rc;; esac
