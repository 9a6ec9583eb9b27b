# Mixtral 2-layer mbs 4: overlap on/off and a kernel trace (regression hunt)
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
for ov in off on; do
  timeout -k 10 500 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --mbs 4 --ga 4 --steps 4 --warmup 2 --optimizer-overlap $ov --no-telemetry >> $O/mbs4.jsonl 2>> $O/mbs4.err
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mbs4 -o run -- python3 bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --mbs 4 --ga 4 --steps 2 --warmup 1 --no-telemetry --comm-sweep off --mesh-sweep off > $O/prof_mbs4.log 2>&1
echo "== done"
