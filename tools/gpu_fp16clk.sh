#!/bin/bash
# Effective clock (GRBM_GUI_ACTIVE / 8 / kernel time) of the headline GEMMs in fp16 vs bf16: the same kernels run at
# different clocks under the board's power limit (fp16 operands toggle more multiplier bits than bf16).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for D in fp16 bf16; do
  timeout -k 10 400 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/clk_$D -o run --output-format csv -- python3 bench.py --dtype $D --steps 1 --warmup 1 --ga 2 --n-layers 8 --no-telemetry > gpurun_out/clk_$D.log 2>&1 || { tail -20 gpurun_out/clk_$D.log; exit 1; }
  ls gpurun_out/clk_$D
done
timeout -k 10 120 python3 tools/grouped_pmc_probe.py > gpurun_out/grouped_probe.log 2>&1 || { tail -20 gpurun_out/grouped_probe.log; exit 1; }
cat gpurun_out/grouped_probe.log | tail -2
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/grouped_pmc -o run --output-format csv -- python3 tools/grouped_pmc_probe.py > gpurun_out/grouped_pmc.log 2>&1 || { tail -20 gpurun_out/grouped_pmc.log; exit 1; }
