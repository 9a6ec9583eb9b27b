# overlapped optimizer on / off for the Llama headline and the Mixtral 2-layer bench at HEAD, alternating on one box
cd "$GRAFT_REPO_ROOT"
O=$GRAFT_REPO_ROOT/gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
for i in 1 2; do
  for ov in off on; do
    timeout -k 10 600 python bench.py --steps 4 --warmup 1 --no-telemetry --optimizer-overlap $ov 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('llama', '$ov', d['value'])" >> $O/overlap_onoff.txt; rc=$?; fatal $rc llama
  done
done
for i in 1 2 3; do
  for ov in off on; do
    timeout -k 10 400 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 8 --warmup 2 --no-telemetry --optimizer-overlap $ov 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('mixtral', '$ov', d['value'])" >> $O/overlap_onoff.txt; rc=$?; fatal $rc mixtral
  done
done
cat $O/overlap_onoff.txt
