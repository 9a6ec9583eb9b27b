# Round 6: kernel statistics of the Mixtral 2-layer bench at HEAD (5 timed steps under rocprofv3).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/profmx
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06/profmx -o run -- \
    python3 -u bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 5 --warmup 2 \
    > gpurun_out/r06/profmx/bench.json 2> gpurun_out/r06/profmx/bench.err
rc=$?; echo "prof rc=$rc"; cut -c1-200 gpurun_out/r06/profmx/bench.json
rm -f $(find gpurun_out/r06/profmx -name "*kernel_trace.csv")
exit $rc
