# Round 6 validation: smoke, the GPU suite, the GPU suite under the stream-ordering audit, the headline bench,
# and the Mixtral EP = 8 spot drill with the supervisor-reserved snapshot (notice at step 1).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/val
export TMPDIR=/tmp
chk() { local rc=$1 name=$2; echo "$name rc=$rc"; case $rc in 0|1) return 0;; *) exit $rc;; esac; }
timeout -k 10 300 python -u -c "import __graft_entry__ as e; e.smoke()" > gpurun_out/r06/val/smoke.log 2>&1
chk $? smoke; tail -1 gpurun_out/r06/val/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r06/val/pytest_gpu.log 2>&1
chk $? pytest_gpu; tail -1 gpurun_out/r06/val/pytest_gpu.log; grep -E "FAILED|ERROR" gpurun_out/r06/val/pytest_gpu.log | head
DLGM_STREAM_AUDIT=1 timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r06/val/pytest_gpu_audit.log 2>&1
chk $? pytest_gpu_audit; tail -1 gpurun_out/r06/val/pytest_gpu_audit.log; grep -E "FAILED|ERROR" gpurun_out/r06/val/pytest_gpu_audit.log | head
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/val/bench.json 2> gpurun_out/r06/val/bench.err
chk $? bench; cut -c1-300 gpurun_out/r06/val/bench.json
DRILLS=spot_reserved TAG=r06 timeout -k 10 900 bash tools/gpu_drills_mixtral.sh > gpurun_out/r06/val/drill.log 2>&1
chk $? drill; tail -c 1500 gpurun_out/r06/val/drill.log
