# Round 6: the overlap model again with the CU-free link delay (hipLaunchHostFunc), plus compute-stream occupancy of
# the 8B reference-knob config at 0 / 350 GB/s; then the Mixtral EP = 8 spot drill with the supervisor-reserved snapshot.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/ovl3
export TMPDIR=/tmp
chk() { local rc=$1 name=$2; echo "$name rc=$rc"; case $rc in 0|1) return 0;; *) exit $rc;; esac; }
for g in 0 350; do
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/ovl$g -o ovl -- python -u tools/shadow_rank.py \
      --model llama3-8b --world 8 --rank 0 --ga 4 --steps 1 --warmup 1 --async-comm --live-params 1e9 \
      --reuse-distance 1e9 --local-grads on --link-gbps $g > gpurun_out/r06/ovl3/trace_$g.log 2>&1
  chk $? trace_$g
  python tools/trace_overlap.py /tmp/ovl$g/ovl_kernel_trace.csv --last-step --out gpurun_out/r06/ovl3/summary_$g.json | head -12
done
timeout -k 10 1000 python -u tools/overlap_model.py --out gpurun_out/r06/ovl3/zero3_overlap_model.json \
    > gpurun_out/r06/ovl3/overlap_model.log 2>&1
chk $? overlap; grep "\[overlap\]" gpurun_out/r06/ovl3/overlap_model.log
