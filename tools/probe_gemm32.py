"""Probe: bf16 x bf16 -> fp32 GEMM with accumulation (torch mm.dtype_out / addmm.dtype_out on ROCm)."""
import torch, time
dev = "cuda"
T, D, F = 8192, 4096, 28672
dy = torch.randn(T, F, device=dev, dtype=torch.bfloat16)
x = torch.randn(T, D, device=dev, dtype=torch.bfloat16)
out16 = torch.empty(F, D, device=dev, dtype=torch.bfloat16)
out32 = torch.zeros(F, D, device=dev, dtype=torch.float32)
ref = (dy.float().t() @ x.float())
def t(fn, n=10):
    fn(); torch.cuda.synchronize(); s = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - s) / n * 1e3
print("bf16 out mm ms", t(lambda: torch.mm(dy.t(), x, out=out16)))
try:
    print("fp32 out mm.dtype_out ms", t(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32, out=out32)))
    print("  err", float((out32 - ref).abs().max() / ref.abs().max()))
except Exception as e:
    print("mm.dtype_out FAIL", str(e)[:300])
try:
    out32.zero_()
    torch.addmm(out32, dy.t(), x, beta=1.0, out_dtype=torch.float32, out=out32)
    torch.addmm(out32, dy.t(), x, beta=1.0, out_dtype=torch.float32, out=out32)
    print("  addmm acc err", float((out32 - 2 * ref).abs().max() / (2 * ref).abs().max()))
    print("fp32 addmm beta=1 ms", t(lambda: torch.addmm(out32, dy.t(), x, beta=1.0, out_dtype=torch.float32, out=out32)))
except Exception as e:
    print("addmm.dtype_out FAIL", str(e)[:300])
acc = torch.zeros(F * D, device=dev)
import sys; sys.path.insert(0, '.')
from distributed_llm_training_gpu_manager_amd import ops
print("separate accumulate ms", t(lambda: ops.accumulate_(acc, out16.view(-1), 1.0, 1.0)))
