#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
nproc; free -g | head -2
timeout -k 10 300 python -u tools/probe_restore.py 16 256 > gpurun_out/probe_restore.json 2> gpurun_out/probe_restore.err
rc=$?; rm -f /dev/shm/dlgm-probe-restore.bin; cat gpurun_out/probe_restore.json; exit $rc
