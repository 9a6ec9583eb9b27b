set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mix_d -o run -- python3 bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 2 --warmup 1 --no-telemetry --comm-sweep off --mesh-sweep off > $O/prof_mix_d.log 2>&1
echo done
