#!/usr/bin/env python3
"""Round 6 probe: the LM head's weight gradient over a step's micro-batches -- one grad_mm per micro-batch (the fp32
gradient read and written GA times) vs ONE grad_mm over the concatenated micro-batches (K = GA x tokens), exactly as
ops.gemm.grad_mm issues them (operand plan + transposes included). Mixtral-8x7B head (V 32000, T 4096, GA 4) and the
Llama-3-8B head (V 128256, T 8192, GA 8). Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from distributed_llm_training_gpu_manager_amd.ops.gemm import grad_mm  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1000.0  # us


def case(V, d, T, ga):
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    dl = (torch.randn(ga * T, V, device=dev, generator=g) * 1e-3).to(torch.bfloat16)
    hn = torch.randn(ga * T, d, device=dev, generator=g).to(torch.bfloat16)
    gw = torch.zeros(V, d, device=dev)

    def per_micro():
        for i in range(ga):
            grad_mm(gw, dl[i * T:(i + 1) * T].t(), hn[i * T:(i + 1) * T], i > 0)

    def once():
        grad_mm(gw, dl.t(), hn, False)

    per_micro()
    ref = gw.clone()
    once()
    rel = float((gw - ref).abs().max() / ref.abs().max())
    flop = 2.0 * ga * T * V * d
    a, b = timeit(per_micro), timeit(once)
    return {"V": V, "T": T, "ga": ga, "per_micro_us": round(a, 1), "once_us": round(b, 1),
            "per_micro_PF": round(flop / a / 1e9, 3), "once_PF": round(flop / b / 1e9, 3), "max_rel_diff": rel}


def main():
    print(json.dumps({"mixtral_head": case(32000, 4096, 4096, 4), "llama3_8b_head": case(128256, 4096, 8192, 8)}),
          flush=True)


if __name__ == "__main__":
    main()
