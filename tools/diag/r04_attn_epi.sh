set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_numerics.py -m gpu -x -q --timeout 200 --timeout-method thread -k "flash or attention or attn or llama" > $O/pytest_attn_epi.log 2>&1 || { tail -30 $O/pytest_attn_epi.log; exit 1; }
tail -1 $O/pytest_attn_epi.log
timeout -k 10 300 python tools/bench_kernels.py > $O/bench_kernels_attn_epi.json 2> $O/bench_kernels_attn_epi.err
python3 -c "import json; d=json.load(open('$O/bench_kernels_attn_epi.json')); print({k: d[k] for k in ('flash_fwd','flash_bwd','ab_fwd','ab_bwd')})"
