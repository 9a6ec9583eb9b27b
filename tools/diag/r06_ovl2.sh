# Round 6: why does the 8B reference-knob shadow rank lose ~9 % at 350 GB/s modelled xGMI? Kernel traces at 0 and 350
# GB/s (GA 4, 1 warmup + 1 step), analysed over the last step; then step times with a deeper gather run-ahead / prefetch.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/ovl2
export TMPDIR=/tmp
chk() { local rc=$1 name=$2; echo "$name rc=$rc"; case $rc in 0|1) return 0;; *) exit $rc;; esac; }
for g in 0 350; do
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/ovl$g -o ovl -- python -u tools/shadow_rank.py \
      --model llama3-8b --world 8 --rank 0 --ga 4 --steps 1 --warmup 1 --async-comm --live-params 1e9 \
      --reuse-distance 1e9 --local-grads on --link-gbps $g > gpurun_out/r06/ovl2/trace_$g.log 2>&1
  chk $? trace_$g
  python tools/trace_overlap.py /tmp/ovl$g/ovl_kernel_trace.csv --last-step --out gpurun_out/r06/ovl2/summary_$g.json | head -14
done
for kw in "gather_inflight_limit=16" "prefetch_bucket_size=1.5e9" "gather_inflight_limit=16,prefetch_bucket_size=1.5e9"; do
  timeout -k 10 400 python -u tools/shadow_rank.py --model llama3-8b --world 8 --rank 0 --ga 8 --steps 3 --warmup 1 \
      --async-comm --live-params 1e9 --reuse-distance 1e9 --local-grads on --link-gbps 350 --engine-kw "$kw" \
      --out gpurun_out/r06/ovl2/kw_$kw.json > gpurun_out/r06/ovl2/kw.log 2>&1
  chk $? "kw $kw"; grep "step " gpurun_out/r06/ovl2/kw.log | tail -3
done
