# Round 5 flake A/B: the round-4 failing selection (every engine of test_shadow_async_gpu.py with the then-default
# overlapped optimizer, then the Mixtral EP-4 overlapped-optimizer test with no warm-up run) with
#   pool      -- streams drawn from torch's round-robin pool, as in round 4 (DLGM_STREAM_POOL=1)
#   dedicated -- every named stream its own HIP stream (utils/streams.py, the default)
# RUNS=N repeats each arm.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/digest
sed -i 's/scheduler="constant", grad_clip=1.0)$/scheduler="constant", grad_clip=1.0, optimizer_overlap=True)/' tests/test_shadow_async_gpu.py
grep -c 'grad_clip=1.0, optimizer_overlap=True)' tests/test_shadow_async_gpu.py
K='swiglu or moe or mixtral or expert or mlp'
for arm in ${ARMS:-pool dedicated}; do
  for r in $(seq 1 ${RUNS:-1}); do
    pool=0; [ "$arm" = pool ] && pool=1
    DLGM_STREAM_POOL=$pool timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
        -p no:cacheprovider -k "$K" > gpurun_out/digest/ab_${arm}_$r.txt 2>&1; rc=$?
    echo "arm $arm run $r rc=$rc: $(grep -E 'passed|failed' gpurun_out/digest/ab_${arm}_$r.txt | tail -1)"
    case $rc in 0|1) ;; *) exit $rc;; esac
  done
done
