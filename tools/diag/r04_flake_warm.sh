# The warm-up A/B behind the note in test_overlapped_optimizer_waits_per_group. Run with the test temporarily
# given a DIAG_WARM switch: same = an identical engine run first, llama = a llama-tiny run first, sync = a device sync + 2 s
# sleep, none = as is. Result (round 4): same / llama pass, sync / none fail.
cd "$GRAFT_REPO_ROOT"
for w in same llama sync none; do
  DIAG_WARM=$w timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "swiglu or moe or mixtral or expert or mlp" > gpurun_out/warm_$w.txt 2>&1; rc=$?
  case $rc in 124|134|137|139) echo fatal; exit $rc;; esac
  echo "$w: $(grep -E 'passed|failed' gpurun_out/warm_$w.txt | tail -1)"
done
