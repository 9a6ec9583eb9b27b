# Round 6: the Mixtral EP = 8 spot drill with the duty-cycled background registration (first step vs the preparation).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/val4
export TMPDIR=/tmp
chk() { local rc=$1 name=$2; echo "$name rc=$rc"; case $rc in 0|1) return 0;; *) exit $rc;; esac; }
DRILLS=spot_reserved TAG=r06 timeout -k 10 900 bash tools/gpu_drills_mixtral.sh > gpurun_out/r06/val4/drill.log 2>&1
chk $? drill; python3 -c "
import json; d=json.load(open('gpurun_out/drills_mixtral_8x7b_ep8_shadow_r06.json'))['spot_reserved']
print(json.dumps({k: d.get(k) for k in ('emergency_ckpt','margin_to_notice_window_s','emergency_record','ckpt_prepare','startup_timeline')})[:1500])"
