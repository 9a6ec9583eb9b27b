#!/usr/bin/env python3
"""Per-kernel micro-benchmarks at Llama-3-8B training shapes (T = 8192 tokens).

Reports achieved HBM bandwidth (memory-bound kernels) or TFLOP/s (attention), and
the PyTorch reference alternative where one exists (torch SDPA for attention,
eager ops for the elementwise kernels) so every number has a comparison point.
Random (not zero) data everywhere (MI355X clocks run higher on zeros).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_training_gpu_manager_amd import ops  # noqa: E402
from distributed_llm_training_gpu_manager_amd.ops import attention as A  # noqa: E402


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters / 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    dev = "cuda"
    T, D, F_, V = args.seq, 4096, 14336, 128256
    H, Hk, hd = 32, 8, 128
    res = {}
    bf = torch.bfloat16

    def want(k):
        return not args.only or k in args.only.split(",")

    if want("rmsnorm"):
        x = torch.randn(T, D, device=dev, dtype=bf)
        r = torch.randn(T, D, device=dev, dtype=bf)
        w = torch.randn(D, device=dev, dtype=bf)
        t = timeit(lambda: ops.rmsnorm_fwd(x, w, 1e-5, residual=r))
        res["add_rmsnorm_fwd"] = {"ms": t * 1e3, "GBps": 4 * T * D * 2 / t / 1e9}
        y, h, rs = ops.rmsnorm_fwd(x, w, 1e-5, residual=r)
        dw = torch.empty(D, device=dev)
        t = timeit(lambda: ops.rmsnorm_bwd(x, h, w, rs, dw, dres=r))
        res["rmsnorm_bwd"] = {"ms": t * 1e3, "GBps": 4 * T * D * 2 / t / 1e9}
        t = timeit(lambda: F.rms_norm((x.float() + r.float()).to(bf), (D,), w, 1e-5))
        res["torch_add_rmsnorm_fwd"] = {"ms": t * 1e3}
    if want("rope"):
        qkv = torch.randn(T, (H + 2 * Hk) * hd, device=dev, dtype=bf)
        cos, sin = ops.rope_tables(hd, T, 5e5, dev)
        t = timeit(lambda: ops.rope_(qkv, cos, sin, H + Hk, hd, T))
        res["rope"] = {"ms": t * 1e3, "GBps": 2 * T * (H + Hk) * hd * 2 / t / 1e9}
    if want("swiglu"):
        gu = torch.randn(T, 2 * F_, device=dev, dtype=bf)
        dy = torch.randn(T, F_, device=dev, dtype=bf)
        t = timeit(lambda: ops.swiglu_fwd(gu))
        res["swiglu_fwd"] = {"ms": t * 1e3, "GBps": 3 * T * F_ * 2 / t / 1e9}
        t = timeit(lambda: ops.swiglu_bwd(dy, gu))
        res["swiglu_bwd"] = {"ms": t * 1e3, "GBps": 5 * T * F_ * 2 / t / 1e9}
    if want("ce"):
        logits = torch.randn(T, V, device=dev, dtype=bf)
        labels = torch.randint(0, V, (T,), device=dev)
        t = timeit(lambda: ops.cross_entropy_fwd_bwd_(logits, labels, 1.0 / T), iters=5)
        res["cross_entropy_fwd_bwd"] = {"ms": t * 1e3, "GBps": 3 * T * V * 2 / t / 1e9}
    if want("adamw"):
        n = 1 << 30
        p, m, v, g = (torch.randn(n, device=dev) for _ in range(4))
        p16 = torch.empty(n, device=dev, dtype=bf)
        st = torch.zeros(2, device=dev)
        t = timeit(lambda: ops.grad_stats([g], st), iters=5)
        res["grad_stats_1G"] = {"ms": t * 1e3, "GBps": n * 4 / t / 1e9}
        t = timeit(lambda: ops.adamw_step_(p, m, v, g, p16, st, lr=1e-4, beta1=0.9, beta2=0.999, eps=1e-8,
                                            weight_decay=0.01, step=2, max_norm=1.0), iters=5)
        res["adamw_1G"] = {"ms": t * 1e3, "GBps": n * (4 * 7 + 2) / t / 1e9}
        del p, m, v, g
    if want("attn"):
        B = 1
        qkv = torch.randn(B, T, (H + 2 * Hk) * hd, device=dev, dtype=bf)
        q = qkv[..., : H * hd].view(B, T, H, hd)
        k = qkv[..., H * hd:(H + Hk) * hd].view(B, T, Hk, hd)
        v = qkv[..., (H + Hk) * hd:].view(B, T, Hk, hd)
        flops_f = 4 * B * H * T * T * hd / 2
        t = timeit(lambda: ops.flash_attn_fwd(q, k, v, None, True), iters=10)
        res["flash_fwd"] = {"ms": t * 1e3, "TFLOPs": flops_f / t / 1e12}
        o, lse = ops.flash_attn_fwd(q, k, v, None, True)
        do = torch.randn_like(o)
        t = timeit(lambda: ops.flash_attn_bwd(do, q, k, v, o, lse, None, True), iters=5)
        res["flash_bwd"] = {"ms": t * 1e3, "TFLOPs": 2.5 * flops_f / t / 1e12}
        qh, kh, vh = (x.permute(0, 2, 1, 3).contiguous() for x in (q, k, v))
        try:
            t = timeit(lambda: F.scaled_dot_product_attention(qh, kh, vh, is_causal=True, enable_gqa=True), iters=10)
            res["torch_sdpa_fwd"] = {"ms": t * 1e3, "TFLOPs": flops_f / t / 1e12}
            qh.requires_grad_(); kh.requires_grad_(); vh.requires_grad_()
            dob = do.permute(0, 2, 1, 3)

            def fb():
                oo = F.scaled_dot_product_attention(qh, kh, vh, is_causal=True, enable_gqa=True)
                oo.backward(dob)
            t = timeit(fb, iters=5)
            res["torch_sdpa_fwd_bwd"] = {"ms": t * 1e3, "TFLOPs": 3.5 * flops_f / t / 1e12}
        except Exception as e:  # pragma: no cover
            res["torch_sdpa"] = {"error": str(e)[:200]}
    if want("attn_ab"):
        # A/B of kernel variants switched by environment variables, interleaved rounds in ONE process
        # (cdna_hip_programming.md §5.4 rule 24): medians and minima per variant
        B = 1
        qkv = torch.randn(B, T, (H + 2 * Hk) * hd, device=dev, dtype=bf)
        q = qkv[..., : H * hd].view(B, T, H, hd)
        k = qkv[..., H * hd:(H + Hk) * hd].view(B, T, Hk, hd)
        v = qkv[..., (H + Hk) * hd:].view(B, T, Hk, hd)
        flops_f = 4 * B * H * T * T * hd / 2
        o, lse = ops.flash_attn_fwd(q, k, v, None, True)
        do = torch.randn_like(o)
        # variants: DLGM_AB="label:fwd|bwd:VAR=val,..." (a label with no VAR=val runs the defaults)
        variants = {"fwd": ("fwd", {}), "bwd": ("bwd", {})}
        for item in os.environ.get("DLGM_AB", "").split(","):
            parts = item.split(":")
            if len(parts) == 3 and "=" in parts[2]:
                var, val = parts[2].split("=", 1)
                variants[parts[0]] = (parts[1], {var: val})
        samples = {n: [] for n in variants}
        for _ in range(5):
            for n, (kind, envs) in variants.items():
                old = {e: os.environ.get(e) for e in envs}
                os.environ.update(envs)
                if kind == "fwd":
                    t = timeit(lambda: ops.flash_attn_fwd(q, k, v, None, True), iters=10)
                else:
                    t = timeit(lambda: ops.flash_attn_bwd(do, q, k, v, o, lse, None, True), iters=5)
                for e, val in old.items():
                    if val is None:
                        os.environ.pop(e, None)
                    else:
                        os.environ[e] = val
                samples[n].append(t)
        for n, ts in samples.items():
            ts = sorted(ts)
            fl = flops_f if variants[n][0] == "fwd" else 2.5 * flops_f
            res["ab_" + n] = {"median_ms": ts[len(ts) // 2] * 1e3, "min_ms": ts[0] * 1e3,
                              "TFLOPs_median": fl / ts[len(ts) // 2] / 1e12}
    if want("gemm"):
        a = torch.randn(T, D, device=dev, dtype=bf)
        w = torch.randn(2 * F_, D, device=dev, dtype=bf)
        t = timeit(lambda: torch.mm(a, w.t()))
        res["gemm_gate_up_8192x28672x4096"] = {"ms": t * 1e3, "TFLOPs": 2 * T * D * 2 * F_ / t / 1e12}
    print(json.dumps({k: {kk: round(vv, 3) if isinstance(vv, float) else vv for kk, vv in v.items()}
                      for k, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
