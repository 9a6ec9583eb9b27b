#!/bin/bash
# One GPU session: build check, kernel/engine tests, smoke, kernel micro-bench, headline bench, rocprof.
# Each GPU step has its own time limit; steps are chained with && so a failure ends the session.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
MODE=${1:-all}
STEPS=${BENCH_STEPS:-3}
run() { echo "== $*" >&2; "$@"; }
if [ "$MODE" = "all" ] || [ "$MODE" = "test" ]; then
  run timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  tail -30 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  run timeout -k 10 300 python __graft_entry__.py smoke 2>&1 | tee gpurun_out/smoke.log || exit 1
fi
if [ "$MODE" = "all" ] || [ "$MODE" = "kbench" ]; then
  run timeout -k 10 300 python tools/bench_kernels.py > gpurun_out/bench_kernels.json 2> gpurun_out/bench_kernels.err || { cat gpurun_out/bench_kernels.err | tail -20; exit 1; }
  cat gpurun_out/bench_kernels.json
fi
if [ "$MODE" = "all" ] || [ "$MODE" = "bench" ]; then
  run timeout -k 10 900 python bench.py --steps $STEPS --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
if [ "$MODE" = "all" ] || [ "$MODE" = "prof" ]; then
  cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
  run timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/prof.log 2>&1 || { tail -30 gpurun_out/prof.log; exit 1; }
  find gpurun_out/prof -name "*kernel_stats.csv" | head -3
fi
echo "== done"
