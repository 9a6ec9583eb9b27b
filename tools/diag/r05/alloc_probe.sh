# Round 5: the 70B rank-scale first steps (rank 0 of 8, shadow) issue for 6-13 s on the host and the caching
# allocator retries once per step at ~283 GiB reserved. A/B: default allocator, expandable segments, more headroom.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/digest
rm -f /dev/shm/dlgm-ckpt-* 2>/dev/null
run() {
  name=$1; shift
  timeout -k 10 300 python -u tools/probe_startup.py --steps ${STEPS:-5} --per-unit 0 --ckpt-tier shm "$@" \
      --out gpurun_out/digest/st_$name.json > gpurun_out/digest/st_$name.txt 2>&1; rc=$?
  echo "$name rc=$rc"; rm -f /dev/shm/dlgm-ckpt-* /dev/shm/probe* 2>/dev/null
  return $rc
}
for arm in ${ARMS:-default expand head16}; do
  case $arm in
    default) run default || exit $? ;;
    expand) PYTORCH_HIP_ALLOC_CONF=expandable_segments:True PYTORCH_CUDA_ALLOC_CONF=expandable_segments:True \
              run expand || exit $? ;;
    head16) run head16 --headroom 0.16 || exit $? ;;
    head22) run head22 --headroom 0.22 || exit $? ;;
  esac
done
