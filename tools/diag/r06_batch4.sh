# Round 6: stored-dS backward with the transpose after the dV/dK MFMAs (A/B kernel stats), and a kernel trace of the
# Llama-3-8B reference-knob shadow rank at 350 GB/s modelled xGMI (where is link time exposed?).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
chk() { local rc=$1 name=$2; echo "$name rc=$rc"; case $rc in 0|1) return 0;; *) exit $rc;; esac; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_kernels_gpu.py -k "flash or attention" > gpurun_out/r06/attn_tests4.log 2>&1
chk $? attn_tests; tail -1 gpurun_out/r06/attn_tests4.log
DLGM_AB=rec:bwd:DLGM_ATTN_BWD=recompute timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $GRAFT_REPO_ROOT/gpurun_out/r06/prof_attn4 -o attn -- python -u tools/bench_kernels.py --only attn_ab \
    > gpurun_out/r06/attn_ab4.log 2>&1
chk $? attn_prof; grep -A2 '"ab_' gpurun_out/r06/attn_ab4.log | grep median
head -8 gpurun_out/r06/prof_attn4/attn_kernel_stats.csv | cut -d, -f1-4
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/ovl -o ovl -- python -u tools/shadow_rank.py \
    --model llama3-8b --world 8 --rank 0 --ga 4 --steps 1 --warmup 1 --async-comm --live-params 1e9 \
    --reuse-distance 1e9 --local-grads on --link-gbps 350 > gpurun_out/r06/ovl_trace.log 2>&1
chk $? ovl_trace
python tools/trace_overlap.py /tmp/ovl/ovl_kernel_trace.csv --skip-s 0 --out gpurun_out/r06/ovl_trace_summary.json | head -40
# the corrected audit over the round-4 tree's shadow-async suite (the mesh cases need the protocol exemption HEAD has)
(cd _bisect/r04 && DLGM_STREAM_AUDIT=1 timeout -k 10 400 python -u -m pytest -v --timeout 250 --timeout-method thread \
    -p no:cacheprovider -m gpu tests/test_shadow_async_gpu.py -k "not mesh" > $GRAFT_REPO_ROOT/gpurun_out/r06/audit_r04_v3.log 2>&1)
chk $? audit_r04; tail -1 gpurun_out/r06/audit_r04_v3.log
