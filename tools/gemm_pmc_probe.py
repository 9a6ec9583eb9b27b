"""One GEMM shape, MFMA kernel vs hipBLASLt, a few launches each (for rocprofv3 --pmc passes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_training_gpu_manager_amd.ops import gemm as G  # noqa: E402
from distributed_llm_training_gpu_manager_amd.ops import gemm_mfma as gm  # noqa: E402

T, O, I = 8192, 6144, 4096
x = torch.randn(T, I, device="cuda").to(torch.bfloat16)
W = (torch.randn(O, I, device="cuda") * 0.02).to(torch.bfloat16)
dy = torch.randn(T, O, device="cuda").to(torch.bfloat16)
out = torch.empty(T, O, device="cuda", dtype=torch.bfloat16)
wg = torch.zeros(O, I, device="cuda")
for _ in range(5):
    gm.mfma_mm(out, x, W.t())
    G.mm(x, W.t())
    gm.mfma_mm(wg, dy.t(), x, acc=True)
    G.grad_mm(wg, dy.t(), x, True)
torch.cuda.synchronize()
print("done")
