# Round 5: (1) two fresh 70B rank-scale engine constructions back to back, no shm file (is the 4.6 s engine_s of a
# later process GPU-side?), (2) the 70B SIGKILL drill, (3) the Mixtral EP=8 spot + SIGKILL drills.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/digest
rm -f /dev/shm/dlgm-ckpt-* 2>/dev/null
for i in 1 2; do
  timeout -k 10 200 python -u tools/probe_startup.py --steps 1 --per-unit 0 --out gpurun_out/digest/engine_twice_$i.json \
      > gpurun_out/digest/engine_twice_$i.txt 2>&1 || exit $?
  python -c "import json;d=json.load(open('gpurun_out/digest/engine_twice_$i.json'));print('engine_s',d['engine_s'],'step',d['steps'][0]['step_s'])"
done
TAG=${TAG:-r05_v1} timeout -k 10 1000 bash tools/gpu_drills_70b.sh > gpurun_out/drill70_v1.txt 2>&1
rc=$?; echo "70b rc=$rc"; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r05_v1} timeout -k 10 1000 bash tools/gpu_drills_mixtral.sh > gpurun_out/drillmix_v1.txt 2>&1
rc=$?; echo "mixtral rc=$rc"; exit $rc
