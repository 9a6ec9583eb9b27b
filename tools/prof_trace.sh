#!/bin/bash
# Kernel trace of the headline bench (default GA 8, one warmup + one timed step) -> per-dispatch CSV.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/trace
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/trace -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/trace.log 2>&1
rc=$?; grep '^{' gpurun_out/trace.log | cut -c1-200; ls gpurun_out/trace; exit $rc
