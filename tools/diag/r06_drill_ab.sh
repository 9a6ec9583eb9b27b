# Round 6: the Mixtral EP = 8 spot drill (notice at step 1, supervisor-reserved and pre-faulted snapshot) under several map / page-lock
# settings of the background preparation -- emergency checkpoint time vs the first step of the fresh job.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/drill_ab
export TMPDIR=/tmp
one() {
  local tag=$1; shift
  env "$@" DRILLS=spot_reserved TAG=ab_$tag timeout -k 10 600 bash tools/gpu_drills_mixtral.sh > gpurun_out/r06/drill_ab/$tag.log 2>&1
  local rc=$?
  python3 -c "
import json; d=json.load(open('gpurun_out/drills_mixtral_8x7b_ep8_shadow_ab_$tag.json'))['spot_reserved']
st=(d.get('startup_timeline') or [{}])[0]; pr=(d.get('ckpt_prepare') or [{}])[0]; er=(d.get('emergency_record') or [{}])[0]
print('$tag', json.dumps({'emergency': d.get('emergency_ckpt'), 'first_step_s': st.get('first_step_s'),
  'prep_done_s': pr.get('done_after_start_s'), 'register_s': pr.get('register_s'), 'save_locked_GB': round((er.get('ring') or {}).get('locked_bytes', 0)/1e9, 1)}))" || true
  [ $rc -eq 0 ]
}
one pf_default X=1 && one pf_write DLGM_SHM_MAP=write && one pf_read DLGM_SHM_MAP=read
