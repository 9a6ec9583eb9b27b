# Round 6: the Mixtral EP = 8 spot drill with the default map stages (background: touch; save: populate-write) and the
# runtime GPU tests.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/val5
export TMPDIR=/tmp
chk() { local rc=$1 name=$2; echo "$name rc=$rc"; case $rc in 0|1) return 0;; *) exit $rc;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_runtime.py -m gpu -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r06/val5/pytest_runtime.log 2>&1
chk $? pytest_runtime; tail -1 gpurun_out/r06/val5/pytest_runtime.log
DRILLS=spot_reserved TAG=r06 timeout -k 10 600 bash tools/gpu_drills_mixtral.sh > gpurun_out/r06/val5/drill.log 2>&1
chk $? drill; python3 -c "
import json; d=json.load(open('gpurun_out/drills_mixtral_8x7b_ep8_shadow_r06.json'))['spot_reserved']
st=(d.get('startup_timeline') or [{}])[0]; pr=(d.get('ckpt_prepare') or [{}])[0]; er=(d.get('emergency_record') or [{}])[0]
print(json.dumps({'emergency': d.get('emergency_ckpt'), 'margin': d.get('margin_to_notice_window_s'), 'first_step_s': st.get('first_step_s'),
  'prep_done_s': pr.get('done_after_start_s'), 'save_locked_GB': round((er.get('ring') or {}).get('locked_bytes', 0)/1e9, 1), 'capture_s': er.get('capture_s')}))"
