"""Forward / input-gradient GEMM layouts vs weight storage: W [out, in] (current) or Wt [in, out].

fwd : y[T,out]  = x[T,in] @ W^T      (W stored [out,in]: "TN";  Wt stored [in,out]: "NN")
dX  : dx[T,in]  = dy[T,out] @ W      (W: "NN";                  Wt: dy @ Wt^T "TN")
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
tot = {"W": 0.0, "Wt": 0.0, "best": 0.0}
for name, (N, K) in shapes.items():
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    W = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    Wt = W.t().contiguous()
    fl = 2.0 * T * N * K
    r = {"fwd_W": bench(lambda: torch.mm(x, W.t())), "fwd_Wt": bench(lambda: torch.mm(x, Wt)),
         "dx_W": bench(lambda: torch.mm(dy, W)), "dx_Wt": bench(lambda: torch.mm(dy, Wt.t()))}
    a, b = r["fwd_W"] + r["dx_W"], r["fwd_Wt"] + r["dx_Wt"]
    tot["W"] += a
    tot["Wt"] += b
    tot["best"] += min(a, b)
    print(f"{name:10s} " + " ".join(f"{k}={v:.3f}ms({fl / v / 1e9:.0f}TF)" for k, v in r.items()) +
          f" | W {a:.3f} Wt {b:.3f}", flush=True)
    del x, dy, W, Wt
print("totals", {k: round(v, 3) for k, v in tot.items()})
