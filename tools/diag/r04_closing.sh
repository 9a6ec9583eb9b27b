# round-4 closing record at HEAD: smoke, the driver's headline command, and a kernel-stats profile of a short run
set -e
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke_closing.log 2>&1
tail -2 $O/smoke_closing.log
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_closing.json 2> $O/bench_closing.err
cat $O/bench_closing.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_closing -o run -- python3 bench.py --steps 3 --warmup 1 --no-telemetry > $O/bench_prof_closing.json 2> $O/prof_closing.err
echo done
