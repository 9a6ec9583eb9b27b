# Round 5 closing measurements at HEAD: the GPU suite, the driver's headline command, the Mixtral 2-layer config,
# and the attention PMC passes.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/closing
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/closing/pytest_gpu.log 2>&1
rc=$?; echo "suite rc=$rc: $(grep -E 'passed|failed' gpurun_out/closing/pytest_gpu.log | tail -1)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/closing/bench.log 2>&1
rc=$?; echo "bench rc=$rc: $(grep '^{' gpurun_out/closing/bench.log | cut -c1-200)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --mbs 1 --ga 4 --steps 20 --warmup 3 \
    > gpurun_out/closing/bench_mixtral.log 2>&1
rc=$?; echo "mixtral rc=$rc: $(grep '^{' gpurun_out/closing/bench_mixtral.log | cut -c1-200)"; [ $rc -eq 0 ] || exit $rc
bash tools/pmc_attn.sh > gpurun_out/closing/pmc.log 2>&1; echo "pmc rc=$?"
