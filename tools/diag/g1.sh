set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06
timeout -k 10 300 python -u tools/bench_kernels.py --only attn_ab > gpurun_out/r06/attn_ab_base.log 2>&1 && \
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06/bench_base.json 2> gpurun_out/r06/bench_base.err
