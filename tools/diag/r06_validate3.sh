# Round 6: threaded populate-write map stage -- the runtime GPU tests, the Mixtral EP = 8 spot drill (notice at step 1,
# supervisor-reserved snapshot), and the Mixtral 2-layer bench at HEAD (with its rocprofv3 kernel stats).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/val3
export TMPDIR=/tmp
chk() { local rc=$1 name=$2; echo "$name rc=$rc"; case $rc in 0|1) return 0;; *) exit $rc;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_runtime.py -m gpu -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r06/val3/pytest_runtime.log 2>&1
chk $? pytest_runtime; tail -1 gpurun_out/r06/val3/pytest_runtime.log
DRILLS=spot_reserved TAG=r06 timeout -k 10 900 bash tools/gpu_drills_mixtral.sh > gpurun_out/r06/val3/drill.log 2>&1
chk $? drill; tail -c 1200 gpurun_out/r06/val3/drill.log
timeout -k 10 400 python -u bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 20 --warmup 3 \
    > gpurun_out/r06/val3/bench_mixtral.json 2> gpurun_out/r06/val3/bench_mixtral.err
chk $? bench_mixtral; cut -c1-400 gpurun_out/r06/val3/bench_mixtral.json
