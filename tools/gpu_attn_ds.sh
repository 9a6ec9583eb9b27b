#!/bin/bash
# stored-dS^T attention backward: numerics with DLGM_ATTN_DQ_FROM_DS=1, interleaved timing vs the recompute dQ,
# and per-kernel times of both under rocprofv3 (kernel trace only)
set -o pipefail
cd "$(dirname "$0")/.." && mkdir -p gpurun_out
DLGM_ATTN_DQ_FROM_DS=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_kernels_fp16_gpu.py -x -q -k "attn or attention or flash" --timeout 120 --timeout-method thread > gpurun_out/attn_tests_ds.log 2>&1 || { grep -E "assert|Error|FAILED" gpurun_out/attn_tests_ds.log | head -20; exit 1; }
tail -1 gpurun_out/attn_tests_ds.log
for r in 1 2; do for v in 0 1; do
  echo "from_ds=$v $(DLGM_ATTN_DQ_FROM_DS=$v timeout -k 10 200 python tools/bench_kernels.py --only attn 2>/dev/null | tr -d '\n ')"
done; done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in 0 1; do
  DLGM_ATTN_DQ_FROM_DS=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ds$v -o run --output-format csv -- python3 tools/bench_kernels.py --only attn > gpurun_out/prof_ds$v.log 2>&1 || exit 1
  python3 - "$v" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/prof_ds{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "flash" in r["Name"] or "gqa" in r["Name"]:
        print(sys.argv[1], r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
