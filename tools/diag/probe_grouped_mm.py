#!/usr/bin/env python3
"""torch._grouped_mm on gfx950 (device offsets, one call for all experts) vs the per-expert hipBLASLt loop, on
Mixtral-8x7B expert shapes (8 experts, 8192 routed rows = one 4096-token micro-batch at top-2)."""
import json
import sys
import time

import torch

torch.manual_seed(0)
dev = "cuda"
E, R, D, F = 8, 8192, 4096, 14336
counts = torch.distributions.Multinomial(R, torch.ones(E)).sample().long()
offs = torch.cumsum(counts, 0).to(torch.int32).to(dev)
x = torch.randn(R, D, device=dev, dtype=torch.bfloat16)
w = torch.randn(E, 2 * F, D, device=dev, dtype=torch.bfloat16) * 0.02  # [E, N, K] like w_gate_up
res = {"counts": counts.tolist()}


def timeit(fn, n=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def loop():
    out = torch.empty(R, 2 * F, device=dev, dtype=torch.bfloat16)
    lo = 0
    for e, n in enumerate(counts.tolist()):
        torch.mm(x[lo:lo + n], w[e].t(), out=out[lo:lo + n])
        lo += n
    return out


try:
    g = torch._grouped_mm(x, w.transpose(1, 2), offs=offs)
    ref = loop()
    res["fwd_rel_err"] = float((g.float() - ref.float()).abs().max() / ref.float().abs().max())
    res["grouped_fwd_ms"] = timeit(lambda: torch._grouped_mm(x, w.transpose(1, 2), offs=offs))
except Exception as e:  # noqa: BLE001
    res["grouped_fwd_error"] = repr(e)[:300]
res["loop_fwd_ms"] = timeit(loop)
flops = 2.0 * R * D * 2 * F
for k in ("grouped_fwd_ms", "loop_fwd_ms"):
    if k in res:
        res[k.replace("_ms", "_TF")] = round(flops / res[k] / 1e9, 1)
# weight gradient: dW_e = dy_e^T x_e  (2-D x 2-D with offsets along K)
dy = torch.randn(R, 2 * F, device=dev, dtype=torch.bfloat16)
try:
    gw = torch._grouped_mm(dy.t(), x, offs=offs)  # [E, 2F, D]
    lo = 0
    err = 0.0
    for e, n in enumerate(counts.tolist()):
        r = dy[lo:lo + n].float().t() @ x[lo:lo + n].float()
        err = max(err, float((gw[e].float() - r).abs().max() / r.abs().max()))
        lo += n
    res["wgrad_rel_err"] = err
    res["grouped_wgrad_ms"] = timeit(lambda: torch._grouped_mm(dy.t(), x, offs=offs))
    res["grouped_wgrad_TF"] = round(flops / res["grouped_wgrad_ms"] / 1e9, 1)
except Exception as e:  # noqa: BLE001
    res["grouped_wgrad_error"] = repr(e)[:300]
print(json.dumps(res))
