#!/bin/bash
# Round 6 closing run at HEAD: the full GPU suite (one process), smoke(), the headline bench (driver's flags) and the
# Mixtral 2-layer bench. Stops at the first step that crashes or times out.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/final3
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r06/final3/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc: $(tail -1 gpurun_out/r06/final3/pytest_gpu.log)"
grep -E "^FAILED|^ERROR" gpurun_out/r06/final3/pytest_gpu.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06/final3/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 gpurun_out/r06/final3/smoke.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/final3/bench.json 2> gpurun_out/r06/final3/bench.err
rc=$?; echo "bench rc=$rc: $(cut -c1-160 gpurun_out/r06/final3/bench.json)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 20 --warmup 5 \
  > gpurun_out/r06/final3/bench_mixtral.json 2> gpurun_out/r06/final3/bench_mixtral.err
rc=$?; echo "mixtral rc=$rc: $(cut -c1-160 gpurun_out/r06/final3/bench_mixtral.json)"; exit $rc
