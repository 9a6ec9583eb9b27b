# Round 6: kernel statistics of the headline bench at HEAD (3 timed steps under rocprofv3).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/prof
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06/prof -o run -- \
    python3 -u bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/r06/prof/bench.json 2> gpurun_out/r06/prof/bench.err
rc=$?; echo "prof rc=$rc"; cut -c1-200 gpurun_out/r06/prof/bench.json
find gpurun_out/r06/prof -name "*kernel_stats.csv" | head -3
rm -f $(find gpurun_out/r06/prof -name "*kernel_trace.csv")
exit $rc
