#!/bin/bash
# Full Llama-3-8B drills (NaN, SIGKILL, spot) through the /dev/shm tier, with the restart timeline and the
# step times after the resume (the shm snapshot is page-locked in pieces in the background)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/drill.py --model llama3-8b --seq 8192 --ga 1 --k 3 --save-interval 2 --steps-after 4 \
    --drills nan,sigkill,spot --timeout 280 --keep-last 1 --ckpt-shm on --ckpt-disk 0 \
    --out gpurun_out/drills_llama3_8b_r03.json > gpurun_out/drills_8b_r03.log 2>&1
rc=$?
rm -f /dev/shm/dlgm-ckpt-* 2>/dev/null
tail -c 1500 gpurun_out/drills_8b_r03.log; exit $rc
