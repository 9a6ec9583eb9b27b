cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --ga 2 > gpurun_out/prof.log 2>&1
rc=$?; tail -5 gpurun_out/prof.log; find gpurun_out/prof -name "*stats*"; exit $rc
