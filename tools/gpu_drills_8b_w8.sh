#!/bin/bash
# Config-3 drill at rank scale on one MI355X: rank 0 of an 8-rank Llama-3-8B ZeRO-3 job (--shadow-world 8: true-size
# partitions and gathers, collectives on RCCL-ordered local streams). NaN injected into this rank's gradient at step K
# -> the on-device latch skips the update, the flag rides the step's all-reduced statistics, the job halts (exit 3);
# plus the spot and SIGKILL drills on the same rank (/dev/shm tier).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f /dev/shm/dlgm-ckpt-* 2>/dev/null
timeout -k 10 900 python -u tools/drill.py --model llama3-8b --seq 8192 --ga 1 --k 3 --save-interval 2 \
    --steps-after 1 --drills nan,spot,sigkill --timeout 400 --keep-last 1 --ckpt-shm on --ckpt-disk 0 \
    --extra "--shadow-world 8 --shadow-rank 0 --telemetry-interval 0" \
    --out gpurun_out/drills_llama3_8b_shadow_w8_r04.json > gpurun_out/drills_8b_w8.log 2>&1
rc=$?
rm -f /dev/shm/dlgm-ckpt-* 2>/dev/null
tail -c 3500 gpurun_out/drills_8b_w8.log; exit $rc
