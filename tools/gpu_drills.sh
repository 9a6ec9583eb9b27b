cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
df -h /tmp | tail -1
timeout -k 10 1100 python -u tools/drill.py --model "${DRILL_MODEL:-llama3-1b}" ${DRILL_EXTRA} --seq "${DRILL_SEQ:-8192}" --ga 1 --k 3 --save-interval 2 \
    --drills "${DRILLS:-nan,sigkill,spot}" --timeout 500 --out "gpurun_out/drills_${DRILL_MODEL:-llama3-1b}.json" > gpurun_out/drills.log 2>&1
rc=$?
tail -c 3000 gpurun_out/drills.log; exit $rc
