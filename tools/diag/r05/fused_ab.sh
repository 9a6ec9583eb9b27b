# Round 5: fused AdamW + W^T copy -- GPU tests, then Mixtral 2-layer (and the headline) alternating on / off.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/digest
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread -p no:cacheprovider \
    tests/test_kernels_gpu.py -k "adamw" tests/test_engine_numerics.py::test_fused_optimizer_transpose_is_bit_identical_gpu \
    > gpurun_out/digest/fused_tests.txt 2>&1
rc=$?; echo "tests rc=$rc: $(grep -E 'passed|failed' gpurun_out/digest/fused_tests.txt | tail -1)"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for f in on off; do
    timeout -k 10 200 python -u bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --mbs 1 --ga 4 --steps 10 --warmup 3 \
        --no-telemetry --fused-opt-transpose $f > gpurun_out/digest/fusedab_mix_${f}_$r.log 2>&1 || exit $?
    echo "mix $f run $r: $(grep '^{' gpurun_out/digest/fusedab_mix_${f}_$r.log | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"], d["ms_per_step"], d["extra"]["mfu_vs_2.5PF_dense_bf16"])')"
  done
done
