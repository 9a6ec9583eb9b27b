# HIP-graph replay of the micro-batch loop: numerics tests, then eager vs graph benches on
# launch-bound models (GPT-2-small ZeRO-1 = BASELINE config 1 model; llama-small)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/graphs
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_engine_numerics.py > gpurun_out/graphs/pytest.log 2>&1 &&
for m in gpt2-small llama-small; do
  for g in "" "--hip-graphs"; do
    timeout -k 10 240 python -u bench.py --model $m --seq 1024 --mbs 8 --ga 4 --zero 1 --steps 20 --warmup 2 $g \
        > gpurun_out/graphs/bench_${m}${g:+_graphs}.json 2> gpurun_out/graphs/bench_${m}${g:+_graphs}.err || exit $?
  done
done
rc=$?
tail -5 gpurun_out/graphs/pytest.log; for f in gpurun_out/graphs/*.json; do echo $f; cut -c1-260 $f; done; exit $rc
