cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/digest
RUNS=2 bash tools/diag/r05/bisect_r04.sh; echo "bisect rc=$?"
for i in 1 2 3; do timeout -k 10 120 python -u tools/diag/r05/vram_alloc.py run$i || exit $?; done
rm -f /dev/shm/dlgm-ckpt-* 2>/dev/null
timeout -k 10 300 python -u tools/probe_startup.py --steps 3 --per-unit 0 --out gpurun_out/digest/limiter_70b.json \
    > gpurun_out/digest/limiter_70b.txt 2>&1 || exit $?
python -c "import json;d=json.load(open('gpurun_out/digest/limiter_70b.json'));print('engine',d['engine_s'],[(s['step_s'],s['reserved_GiB'],s['alloc_retries']) for s in d['steps']])"
TAG=r05_v2 timeout -k 10 900 bash tools/gpu_drills_70b.sh > gpurun_out/drill70_v2.txt 2>&1
rc=$?; echo "70b rc=$rc"; exit $rc
