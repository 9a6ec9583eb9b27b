#!/usr/bin/env python3
"""Does aten's bf16 x bf16 -> fp32 mm (out_dtype, beta 0) launch a fill before the GEMM? (kernel trace)"""
import torch

a = torch.randn(4096, 8192, device="cuda", dtype=torch.bfloat16)
b = torch.randn(8192, 4096, device="cuda", dtype=torch.bfloat16)
out = torch.empty(4096, 4096, device="cuda", dtype=torch.float32)
for _ in range(5):
    torch.mm(a, b, out_dtype=torch.float32, out=out)
torch.cuda.synchronize()
for _ in range(5):
    torch.addmm(out, a, b, beta=1.0, out_dtype=torch.float32, out=out)
torch.cuda.synchronize()
print("ok")
