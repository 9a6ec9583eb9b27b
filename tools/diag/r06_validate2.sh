# Round 6 validation after the mesh-heap pool: smoke, the GPU suite under the stream-ordering audit, the headline
# bench, and the Mixtral EP = 8 spot drill through the job registry with the supervisor-reserved snapshot.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/val2
export TMPDIR=/tmp
chk() { local rc=$1 name=$2; echo "$name rc=$rc"; case $rc in 0|1) return 0;; *) exit $rc;; esac; }
timeout -k 10 300 python -u -c "import __graft_entry__ as e; e.smoke()" > gpurun_out/r06/val2/smoke.log 2>&1
chk $? smoke; tail -1 gpurun_out/r06/val2/smoke.log
DLGM_STREAM_AUDIT=1 timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r06/val2/pytest_gpu_audit.log 2>&1
chk $? pytest_gpu_audit; tail -1 gpurun_out/r06/val2/pytest_gpu_audit.log; grep -E "FAILED|ERROR" gpurun_out/r06/val2/pytest_gpu_audit.log | head
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/val2/bench.json 2> gpurun_out/r06/val2/bench.err
chk $? bench; cut -c1-300 gpurun_out/r06/val2/bench.json
DRILLS=spot_reserved TAG=r06 timeout -k 10 900 bash tools/gpu_drills_mixtral.sh > gpurun_out/r06/val2/drill.log 2>&1
chk $? drill; tail -c 1500 gpurun_out/r06/val2/drill.log
