# round-4 batch 4: optimizer-overlap A/B after removing the join from the per-micro-batch expert check
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_numerics.py -m gpu -x -q --timeout 120 --timeout-method thread -k "overlap or mixtral" > $O/pytest_b4.log 2>&1 || { tail -30 $O/pytest_b4.log; exit 1; }
tail -1 $O/pytest_b4.log
for ov in on off on off on off; do
  timeout -k 10 400 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 6 --warmup 2 --optimizer-overlap $ov --no-telemetry >> $O/mixtral_overlap_ab3.jsonl 2>> $O/mixtral_overlap_ab3.err
done
echo "== mixtral done"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_overlap3 -- python3 bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 2 --warmup 1 --optimizer-overlap on --no-telemetry --comm-sweep off --mesh-sweep off > $O/prof_overlap3.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_overlap_llama -- python3 bench.py --n-layers 4 --steps 2 --warmup 1 --optimizer-overlap on --no-telemetry --comm-sweep off --mesh-sweep off > $O/prof_overlap_llama.log 2>&1
echo "== traces done"
