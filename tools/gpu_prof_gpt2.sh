# kernel-time breakdown of the GPT-2-small step (seq 1024, mbs 8, GA 4, ZeRO-1)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_gpt2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gpt2 -o run -- \
    python -u bench.py --model gpt2-small --seq 1024 --mbs 8 --ga 4 --zero 1 --steps 5 --warmup 2 ${GPT2_ARGS:-} \
    > gpurun_out/prof_gpt2/bench.log 2>&1
rc=$?
f=$(find gpurun_out/prof_gpt2 -name '*kernel_stats.csv' | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {100*float(r["TotalDurationNs"])/tot:5.1f}% n={r["Calls"]:>6} {r["Name"][:110]}')
PY
exit $rc
