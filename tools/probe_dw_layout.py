"""Weight-gradient GEMM layout probe: dW[out,in] (+)= dy[T,out]^T @ x[T,in] (fp32 out, beta=1).

(a) as the model calls it (both operands K-strided: hipBLASLt's slow layout)
(b) transpose both operands first so the GEMM sees K-contiguous rows (the forward GEMM's layout)
(c) transpose only dy
"""
import time

import torch


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


T = 8192
shapes = {"wqkv": (6144, 4096), "wo": (4096, 4096), "w_gate_up": (28672, 4096), "w_down": (4096, 14336),
          "lm_head": (128256, 4096)}
tot = {"a": 0.0, "b": 0.0, "c": 0.0, "d": 0.0}
for name, (N, K) in shapes.items():
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    g = torch.zeros(N, K, device="cuda", dtype=torch.float32)
    fl = 2.0 * T * N * K
    fa = lambda: torch.addmm(g, dy.t(), x, beta=1.0, out_dtype=torch.float32, out=g)  # noqa: E731

    def fb():
        dyT = dy.t().contiguous()
        xT = x.t().contiguous()
        torch.addmm(g, dyT, xT.t(), beta=1.0, out_dtype=torch.float32, out=g)

    def fc():
        dyT = dy.t().contiguous()
        torch.addmm(g, dyT, x, beta=1.0, out_dtype=torch.float32, out=g)

    def fd():
        xT = x.t().contiguous()
        torch.addmm(g, dy.t(), xT.t(), beta=1.0, out_dtype=torch.float32, out=g)

    r = {k: bench(f) for k, f in (("a", fa), ("b", fb), ("c", fc), ("d", fd))}
    dyT, xT = dy.t().contiguous(), x.t().contiguous()
    r["b_gemm_only"] = bench(lambda: torch.addmm(g, dyT, xT.t(), beta=1.0, out_dtype=torch.float32, out=g))
    for k in tot:
        tot[k] += r[k]
    print(name, {k: f"{v:.3f}ms {fl / v / 1e9:.0f}TF" for k, v in r.items()}, flush=True)
    # numerics: same result
    g1 = torch.mm(dy.t(), x, out_dtype=torch.float32)
    g2 = torch.mm(dyT, xT.t(), out_dtype=torch.float32)
    print("   max rel diff", float((g1 - g2).abs().max() / g1.abs().max()))
    del dy, x, g, dyT, xT, g1, g2
print("per-layer-set totals ms", {k: round(v, 3) for k, v in tot.items()})
