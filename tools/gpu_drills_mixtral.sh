#!/bin/bash
# Config-5 drills at Mixtral-8x7B rank scale on one MI355X: rank 0 of an 8-rank expert-parallel job (EP = 8: one
# expert per layer on this rank, ZeRO-3 shards of the dense weights) alone on this GPU (--shadow-world 8), with the
# expert token exchange on the device-driven xGMI mesh kernels (shadow mode: every peer slot is this rank's own heap).
# spot: SIGUSR1 at step K -> emergency checkpoint into the /dev/shm tier -> exit 4 -> restore on a fresh process;
# spot_warm: the same with the notice once the snapshot buffer is prepared (--preempt-when-ready);
# sigkill: SIGKILL at step K under the supervisor -> auto-resume -> MTTR and restore breakdown.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f /dev/shm/dlgm-ckpt-* 2>/dev/null
timeout -k 10 1050 python -u tools/drill.py --model mixtral-8x7b --seq ${SEQ:-4096} --ga 1 --k 3 --save-interval 2 \
    --steps-after 1 --drills ${DRILLS:-spot,sigkill} --timeout 480 --keep-last 1 --ckpt-shm on --ckpt-disk 0 \
    --extra "--expert-parallel 8 --shadow-world 8 --shadow-rank 0 --xgmi-mesh on --telemetry-interval 0" \
    --out gpurun_out/drills_mixtral_8x7b_ep8_shadow_${TAG:-r05}.json > gpurun_out/drills_mixtral.log 2>&1
rc=$?
rm -f /dev/shm/dlgm-ckpt-* 2>/dev/null
tail -c 3000 gpurun_out/drills_mixtral.log; exit $rc
