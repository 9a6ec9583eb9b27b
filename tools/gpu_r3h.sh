#!/bin/bash
# w64 forward check + A/B, then the round-3 batch (offload_param NVMe test, 8B shadow sync/async, kernel stats).
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/gpu_r3g.sh && bash tools/gpu_r3f.sh
