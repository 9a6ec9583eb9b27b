"""Round 5: RMSNorm backward time / effective bandwidth at T = 8192 rows for several widths (the library picked by
DLGM_HIP_LIB): widths that are not multiples of 2048 took the wave-per-row kernel at 16 chunks per lane (VGPR
spills) before the guarded row-block variant."""
import json
import sys

import torch

sys.path.insert(0, ".")
from distributed_llm_training_gpu_manager_amd.ops.norm import rmsnorm_bwd, rmsnorm_fwd  # noqa: E402

res = {}
for D in (4096, 5120, 6656, 8192):
    T = 8192
    x = torch.randn(T, D, device="cuda", dtype=torch.bfloat16)
    r = torch.randn(T, D, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(D, device="cuda", dtype=torch.bfloat16)
    y, h, rstd = rmsnorm_fwd(x, w, 1e-5, r)
    dy = torch.randn_like(y)
    dw = torch.zeros(D, device="cuda", dtype=torch.float32)
    for _ in range(3):
        rmsnorm_bwd(dy, h, w, rstd, dw, r)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        rmsnorm_bwd(dy, h, w, rstd, dw, r)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    res[D] = {"us": round(us, 1), "TBps": round(4 * T * D * 2 / us / 1e6, 2)}  # dy, h, dres in; dx out
print(json.dumps(res))
