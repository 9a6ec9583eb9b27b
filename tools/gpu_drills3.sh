#!/bin/bash
# Round-2 drills on one MI355X with the FULL Llama-3-8B (32 layers): the checkpoint snapshot tier lives in
# /dev/shm (the box's scratch disk cannot hold 112 GB of state), keep_last 1.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
df -h /tmp /dev/shm | tail -2
free -g | head -2
timeout -k 10 900 python -u tools/drill.py --model llama3-8b --seq 8192 --ga 1 --k 3 --save-interval 2 \
    --drills nan,sigkill,spot --timeout 280 --keep-last 1 --ckpt-shm on --ckpt-disk 0 \
    --out gpurun_out/drills_llama3_8b_r02.json > gpurun_out/drills_8b.log 2>&1
rc=$?
rm -f /dev/shm/dlgm-ckpt-* 2>/dev/null
tail -c 2500 gpurun_out/drills_8b.log; exit $rc
