# Round 6: the Llama-3-70B config-4 SIGKILL drill and the Llama-3-8B NaN / spot / SIGKILL drills at HEAD (rank 0 of 8
# alone on one MI355X), after this round's checkpoint changes (supervisor-reserved and pre-faulted snapshots, threaded
# populate in saves, duty-cycled background page-locking, leased streams).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=r06 timeout -k 10 1100 bash tools/gpu_drills_70b.sh > /dev/null 2>&1
rc=$?; echo "70b rc=$rc"; python3 -c "
import json; d=json.load(open('gpurun_out/drills_llama3_70b_shadow_w8_r06.json'))
s=d.get('sigkill', {}); print(json.dumps({k: s.get(k) for k in ('status','mttr_s','restore','exit_codes')})[:600])" || true
[ $rc -eq 0 ] || exit $rc
timeout -k 10 950 bash tools/gpu_drills_8b_w8.sh > /dev/null 2>&1
rc=$?; echo "8b rc=$rc"; python3 -c "
import json; d=json.load(open('gpurun_out/drills_llama3_8b_shadow_w8_r04.json'))
print(json.dumps({k: ({kk: v.get(kk) for kk in ('status','mttr_s','emergency_ckpt','exit_codes','trip_step')} if isinstance(v, dict) else v) for k, v in d.items() if k in ('nan','spot','sigkill')})[:1200])" || true
exit $rc
