#!/bin/bash
# dK/dV time with the dS^T stores as built (cur), rewriting one L2-resident block (diagL2), or packed but not
# stored (diagNo): where the stored-dS cost comes from (rocprofv3 kernel stats, DLGM_ATTN_DQ_FROM_DS=1)
set -o pipefail
cd "$(dirname "$0")/../.." && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for lib in cur diagL2 diagNo; do
  DLGM_ATTN_DQ_FROM_DS=1 DLGM_HIP_LIB=$PWD/ab/$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/diag_$lib -o run --output-format csv -- python3 tools/bench_kernels.py --only attn > gpurun_out/diag_$lib.log 2>&1 || exit 1
  python3 - "$lib" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/diag_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "dkdv" in r["Name"] or "dq_kernel" in r["Name"]:
        print(sys.argv[1], r["Name"][:50], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
