# Round 5 closing drills at HEAD: 70B rank-scale SIGKILL (MTTR) and Mixtral EP=8 spot + SIGKILL.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rm -f /dev/shm/dlgm-ckpt-* 2>/dev/null
TAG=${TAG:-r05} timeout -k 10 1000 bash tools/gpu_drills_70b.sh > gpurun_out/drill70_final.txt 2>&1
rc=$?; echo "70b rc=$rc"; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r05} timeout -k 10 1000 bash tools/gpu_drills_mixtral.sh > gpurun_out/drillmix_final.txt 2>&1
rc=$?; echo "mixtral rc=$rc"; exit $rc
