#!/bin/bash
# Config-4 drill at 70B rank scale on one MI355X: rank 0 of an 8-rank Llama-3-70B ZeRO-3 job
# alone on this GPU (--shadow-world 8: true-size partitions, gathers and snapshot; collectives are local copies on
# RCCL-ordered streams), activation checkpointing as in the reference's 70b preset. SIGKILL under the supervisor at
# step K -> auto-resume from the /dev/shm snapshot tier (~123 GB for this rank) -> MTTR and restore breakdown.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f /dev/shm/dlgm-ckpt-* 2>/dev/null
timeout -k 10 1050 python -u tools/drill.py --model llama3-70b --seq ${SEQ:-8192} --ga 1 --k 3 --save-interval 2 \
    --steps-after 1 --drills sigkill --timeout 1000 --keep-last 1 --ckpt-shm on --ckpt-disk 0 \
    --extra "--shadow-world 8 --shadow-rank 0 --activation-checkpointing --telemetry-interval 0 ${EXTRA:-}" \
    --out gpurun_out/drills_llama3_70b_shadow_w8_${TAG:-r05}.json > gpurun_out/drills_70b.log 2>&1
rc=$?
rm -f /dev/shm/dlgm-ckpt-* 2>/dev/null
tail -c 2500 gpurun_out/drills_70b.log; exit $rc
