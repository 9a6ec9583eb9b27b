# Round 6 batch: stored-dS attention (numerics + kernel trace of the A/B), the API launch GPU test, the ZeRO-3
# overlap model (shadow rank 0 of 8 with modelled xGMI time), and the Llama-3-8B API launch record.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
chk() { local rc=$1 name=$2; echo "$name rc=$rc"; case $rc in 0|1) return 0;; *) exit $rc;; esac; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_kernels_gpu.py tests/test_kernels_fp16_gpu.py -k "flash or attention" > gpurun_out/r06/attn_tests3.log 2>&1
chk $? attn_tests; tail -1 gpurun_out/r06/attn_tests3.log
DLGM_AB=rec:bwd:DLGM_ATTN_BWD=recompute timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $GRAFT_REPO_ROOT/gpurun_out/r06/prof_attn3 -o attn -- python -u tools/bench_kernels.py --only attn_ab \
    > gpurun_out/r06/attn_ab3.log 2>&1
chk $? attn_prof; grep -A2 '"ab_' gpurun_out/r06/attn_ab3.log | grep median
timeout -k 10 400 python -u -m pytest -x -v --timeout 350 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_api_launch_gpu.py > gpurun_out/r06/api_test.log 2>&1
chk $? api_test; tail -1 gpurun_out/r06/api_test.log
timeout -k 10 900 python -u tools/api_launch.py --preset llama3-8b --out gpurun_out/r06/api_launch_llama3_8b.json \
    > gpurun_out/r06/api_launch_8b.log 2>&1
chk $? api_8b; tail -2 gpurun_out/r06/api_launch_8b.log
timeout -k 10 1500 python -u tools/overlap_model.py --out gpurun_out/r06/zero3_overlap_model.json \
    > gpurun_out/r06/overlap_model.log 2>&1
chk $? overlap; grep "\[overlap\]" gpurun_out/r06/overlap_model.log
