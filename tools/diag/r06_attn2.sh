# Round 6: stored-dS attention backward -- numerics, then a kernel trace of the interleaved A/B (both variants).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_kernels_gpu.py tests/test_kernels_fp16_gpu.py -k "flash or attention" > gpurun_out/r06/attn_tests2.log 2>&1
rc=$?; echo "attn_tests rc=$rc: $(tail -1 gpurun_out/r06/attn_tests2.log)"; [ $rc -eq 0 ] || exit $rc
DLGM_AB=rec:bwd:DLGM_ATTN_BWD=recompute timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r06/prof_attn -o attn \
    -- python -u tools/bench_kernels.py --only attn_ab > gpurun_out/r06/attn_ab_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; grep -A3 '"ab_' gpurun_out/r06/attn_ab_prof.log | grep median
find gpurun_out/r06/prof_attn -name "*kernel_stats.csv" | head -2
