set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_v8.json 2> gpurun_out/bench_v8.err || { tail -5 gpurun_out/bench_v8.err; exit 1; }
cat gpurun_out/bench_v8.json
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --mbs 2 --ga 4 > gpurun_out/bench_mbs2.json 2> gpurun_out/bench_mbs2.err || { tail -5 gpurun_out/bench_mbs2.err; exit 1; }
cat gpurun_out/bench_mbs2.json
