# the driver's headline command at HEAD, and a 20-step Mixtral run (memory stability with the side streams)
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err
python3 -c "import json; d=json.load(open('$O/bench_driver_cmd.json')); print(d['value'], d['extra']['mem']['peak_GiB'], d['extra']['telemetry']['power_w'] if d['extra'].get('telemetry') else None)"
timeout -k 10 600 python bench.py --model mixtral-8x7b --n-layers 2 --seq 4096 --ga 4 --steps 20 --warmup 5 --no-telemetry > $O/bench_mix20.json 2> $O/bench_mix20.err
python3 -c "import json; d=json.load(open('$O/bench_mix20.json')); print(d['value'], d['extra']['mem']['peak_GiB'])"
