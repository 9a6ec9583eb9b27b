# BASELINE configs 4 and 5 on one MI355X with the real architectures at reduced depth:
#   Mixtral-8x7B (2 layers, 8 experts top-2, EP world 1): nan + sigkill + spot drills
#   Llama-3-70B (1 layer, d8192 / 64H / 8KV / FFN 28672, full vocab): sigkill drill
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
df -h /tmp | tail -1
free -g | head -2
timeout -k 10 560 python -u tools/drill.py --model mixtral-8x7b --n-layers 2 --seq 8192 --ga 1 --k 3 --save-interval 2 \
    --drills nan,sigkill,spot --timeout 250 --out gpurun_out/drills_mixtral.json > gpurun_out/drills_mixtral.log 2>&1 &&
timeout -k 10 400 python -u tools/drill.py --model llama3-70b --n-layers 1 --seq 8192 --ga 1 --k 3 --save-interval 2 \
    --drills sigkill --timeout 250 --out gpurun_out/drills_70b.json > gpurun_out/drills_70b.log 2>&1
rc=$?
tail -c 1500 gpurun_out/drills_mixtral.log; tail -c 1500 gpurun_out/drills_70b.log; exit $rc
