# Round 5 flake bisect, stage 2: the round-4 tree (reproduces: 2 of 2) against the same tree with only the
# dedicated-stream change of 99d00e7 applied (_bisect/r04s), alternating, on the failing selection.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/digest
K='swiglu or moe or mixtral or expert or mlp'
for r in $(seq 1 ${RUNS:-2}); do
  for v in r04 r04s; do
    (cd _bisect/$v && timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
        -p no:cacheprovider -k "$K" > ../../gpurun_out/digest/bisect_${v}_$r.txt 2>&1); rc=$?
    echo "$v run $r rc=$rc: $(grep -E 'passed|failed' gpurun_out/digest/bisect_${v}_$r.txt | tail -1)"
    case $rc in 0|1) ;; *) exit $rc;; esac
  done
done
