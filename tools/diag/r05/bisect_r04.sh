# Round 5 flake bisect: the round-4 tree (3208a31, warm-up removed from its test, built in _bisect/r04) on the
# failing selection, RUNS times; then HEAD with the round-4 pre-state (overlapped optimizer in every engine).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/digest
K='swiglu or moe or mixtral or expert or mlp'
for r in $(seq 1 ${RUNS:-2}); do
  (cd _bisect/r04 && timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
      -p no:cacheprovider -k "$K" > ../../gpurun_out/digest/bisect_r04_$r.txt 2>&1); rc=$?
  echo "r04 run $r rc=$rc: $(grep -E 'passed|failed' gpurun_out/digest/bisect_r04_$r.txt | tail -1)"
  case $rc in 0|1) ;; *) exit $rc;; esac
done
