#!/usr/bin/env python3
"""Where does the weight-gradient GEMM time go on MI355X? (hipBLASLt, best of the top heuristic candidates)

For each Llama-3-8B dW problem (out [n_out, n_in] = dy^T @ x over T tokens) this times:
  layout  NN: both operands with the token (reduction) dim strided, as the model produces them
          A / B: only the dy^T / only the x operand K-contiguous
          TN: both K-contiguous (what a free transpose would give)
  output  fp32 beta=1 (direct accumulation into the gradient), fp32 beta=0, bf16 beta=0
  tokens  T and 2T (two micro-batches concatenated along K)
and prints TFLOP/s per case, so the cost of the fp32 epilogue, of the layout and of K can be separated.

    python tools/probe_dw_cost.py [--tokens 8192] [--topn 32]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_llm_training_gpu_manager_amd import _native  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--topn", type=int, default=32)
    ap.add_argument("--out", default="")
    ap.add_argument("--no-concat", action="store_true", help="skip the 2T (two micro-batches) cases")
    a = ap.parse_args()
    ops = _native.hip_ops()
    dev = torch.device("cuda")
    bf = dict(dtype=torch.bfloat16, device=dev)
    rows = []
    for name, n_out, n_in in (("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)):
        for T in ((a.tokens,) if a.no_concat else (a.tokens, 2 * a.tokens)):
            x = torch.randn(T, n_in, **bf)
            dy = torch.randn(T, n_out, **bf)
            dyT, xT = dy.t().contiguous(), x.t().contiguous().t()
            lay = {"NN": (dy.t(), x), "A": (dyT, x), "B": (dy.t(), xT), "TN": (dyT, xT)}
            for ln, (A, B) in lay.items():
                for on, dt, beta in (("f32b1", torch.float32, 1.0), ("f32b0", torch.float32, 0.0),
                                     ("bf16b0", torch.bfloat16, 0.0)):
                    out = torch.zeros(n_out, n_in, dtype=dt, device=dev)
                    try:
                        res = ops.gemm_lt_tune(out, A, B, beta, a.topn, False, 3)
                    except RuntimeError as e:  # no solution for this combination
                        print(name, T, ln, on, "error", str(e)[:80], flush=True)
                        continue
                    us = float(res[0, 1])
                    tf = 2.0 * n_out * n_in * T / us / 1e6
                    r = {"gemm": name, "tokens": T, "layout": ln, "out": on, "us": round(us, 1),
                         "TF": round(tf, 1), "us_per_8k_tokens": round(us * a.tokens / T, 1)}
                    rows.append(r)
                    print(json.dumps(r), flush=True)
                    del out
            del x, dy, lay
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"device": torch.cuda.get_device_properties(0).gcnArchName, "rows": rows}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
