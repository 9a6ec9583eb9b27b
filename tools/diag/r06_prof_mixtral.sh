# Round 6: kernel statistics of the Mixtral 2-layer bench at HEAD (5 timed steps under rocprofv3), plus the order
# and grid sizes of the fill / transpose kernels of one step (to attribute them).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/profmx3
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06/profmx3 -o run -- \
    python3 -u bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 5 --warmup 2 \
    > gpurun_out/r06/profmx3/bench.json 2> gpurun_out/r06/profmx3/bench.err
rc=$?; echo "prof rc=$rc"; cut -c1-200 gpurun_out/r06/profmx3/bench.json
python3 - <<'EOF'
import csv, glob
f = glob.glob("gpurun_out/r06/profmx3/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
ad = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
lo, hi = ad[-2] + 1, ad[-1] + 1  # the last full step
with open("gpurun_out/r06/profmx3/step_order.txt", "w") as out:
    for r in rows[lo:hi]:
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        out.write(f'{us:9.1f} {r["Grid_Size_X"]:>9} {r["Workgroup_Size_X"]:>5} {r["Kernel_Name"][:120]}\n')
print("step kernels", hi - lo)
EOF
rm -f $(find gpurun_out/r06/profmx3 -name "*kernel_trace.csv")
exit $rc
