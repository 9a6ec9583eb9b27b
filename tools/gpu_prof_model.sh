#!/bin/bash
# Kernel-time breakdown of one bench configuration: tools/gpu_prof_model.sh <tag> <bench.py args...>
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- \
    python -u bench.py "$@" > $out/bench.log 2>&1
rc=$?
grep '^{' $out/bench.log
f=$(find $out -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:22]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {100*float(r["TotalDurationNs"])/tot:5.1f}% n={r["Calls"]:>6} {r["Name"][:100]}')
PY
exit $rc
