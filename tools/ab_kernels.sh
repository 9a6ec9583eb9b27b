#!/bin/bash
# Same-device A/B of kernel builds: bash tools/ab_kernels.sh <bench --only list> <lib1.so> <lib2.so> ...
# Interleaved rounds (lib1, lib2, lib1, lib2, ...) so DVFS / device drift hits every variant alike.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
only=$1; shift
for round in 1 2; do
  for lib in "$@"; do
    echo "== round $round $lib"
    DLGM_HIP_LIB=$PWD/$lib timeout -k 10 300 python tools/bench_kernels.py --only "$only" 2>/dev/null | tr -d '\n ' ; echo
  done
done
