#!/bin/bash
# Llama-3-8B SIGKILL drill only (the /dev/shm tier), with the restart timeline (MTTR breakdown)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DLGM_CKPT_PREPARE=${DLGM_CKPT_PREPARE:-1} timeout -k 10 600 python -u tools/drill.py --model llama3-8b --seq 8192 --ga 1 --k 3 --save-interval 2 --steps-after ${DRILL_AFTER:-0} \
    --drills sigkill --timeout 280 --keep-last 1 --ckpt-shm on --ckpt-disk 0 \
    --out gpurun_out/drill_mttr_8b.json > gpurun_out/drill_mttr_8b.log 2>&1
rc=$?
rm -f /dev/shm/dlgm-ckpt-* 2>/dev/null
tail -c 1500 gpurun_out/drill_mttr_8b.log; exit $rc
