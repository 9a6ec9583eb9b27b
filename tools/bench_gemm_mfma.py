#!/usr/bin/env python3
"""Hand-written MFMA GEMM vs the current engine path on the Llama-3-8B GEMMs (interleaved rounds, one process).

dW (dy^T x, fp32 beta=1): gemm_mfma straight from the token-major operands vs ops.gemm.grad_mm (hipBLASLt with
the layout plan's transposes). Forward (x @ W^T, bf16 out): gemm_mfma vs ops.gemm.mm. Random operands.
"""
import json
import sys
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_llm_training_gpu_manager_amd.ops import gemm as G  # noqa: E402
from distributed_llm_training_gpu_manager_amd.ops import gemm_mfma as gm  # noqa: E402


def timeit(fn, reps=10):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    shapes = {"wqkv": (6144, 4096), "wo": (4096, 4096), "w_gate_up": (28672, 4096), "w_down": (4096, 14336),
              "lm_head": (128256, 4096)}
    dev = "cuda"
    res = {}
    for name, (O, I) in shapes.items():
        dy = torch.randn(T, O, device=dev).to(torch.bfloat16)
        x = torch.randn(T, I, device=dev).to(torch.bfloat16)
        w = torch.zeros(O, I, device=dev)
        W = (torch.randn(O, I, device=dev) * 0.02).to(torch.bfloat16)
        fl = 2.0 * T * O * I
        arms = {
            "dW_mfma": lambda: gm.mfma_mm(w, dy.t(), x, acc=True),
            "dW_engine": lambda: G.grad_mm(w, dy.t(), x, True),
            "fwd_mfma": lambda: gm.mfma_mm(torch.empty(T, O, device=dev, dtype=torch.bfloat16), x, W.t()),
            "fwd_engine": lambda: G.mm(x, W.t()),
        }
        ts = {k: [] for k in arms}
        for _ in range(5):
            for k, f in arms.items():
                ts[k].append(timeit(f))
        r = {}
        for k, v in ts.items():
            v.sort()
            r[k] = {"ms": round(v[len(v) // 2], 3), "TFLOPs": round(fl / (v[len(v) // 2] * 1e-3) / 1e12, 1)}
        # numerics of the dW / forward arms against fp32
        ref = dy.float().t() @ x.float()
        w.zero_()
        gm.mfma_mm(w, dy.t(), x, acc=True)
        r["dW_rel_err"] = float((w - ref).abs().max() / ref.abs().max())
        del ref
        fref = x.float() @ W.float().t()
        o = gm.mfma_mm(torch.empty(T, O, device=dev, dtype=torch.bfloat16), x, W.t())
        r["fwd_rel_err"] = float((o.float() - fref).abs().max() / fref.abs().max())
        del fref, o
        res[name] = r
        print(name, json.dumps(r), flush=True)
        del dy, x, w, W
        torch.cuda.empty_cache()
    print(json.dumps({"T": T, "results": res}))


if __name__ == "__main__":
    main()
