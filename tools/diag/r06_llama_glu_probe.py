#!/usr/bin/env python3
"""Round 6 probe: the Llama-3-8B MLP input gradient at the headline shape (T 8192, d 4096, F 14336) --
(A) hipBLASLt dA = dY @ W_down then the swiglu_bwd kernel (the engine today) vs (B) the MFMA GEMM with the SwiGLU
backward in its epilogue (grouped-M launch with one group), plus each GEMM alone. Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from distributed_llm_training_gpu_manager_amd import ops  # noqa: E402
from distributed_llm_training_gpu_manager_amd.ops import gemm_mfma as gm  # noqa: E402
from distributed_llm_training_gpu_manager_amd.ops.gemm import mm  # noqa: E402


def timeit(fn, reps=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1000.0  # us


def main():
    dev = "cuda"
    T, d, F = 8192, 4096, 14336
    g = torch.Generator(device=dev).manual_seed(0)
    dy = (torch.randn(T, d, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    wt = (torch.randn(F, d, device=dev, generator=g) * 0.02).to(torch.bfloat16)  # W_down^T cache [F, d]
    gu = torch.randn(T, 2 * F, device=dev, generator=g).to(torch.bfloat16)
    offs = torch.tensor([0, T], dtype=torch.int32, device=dev)
    w3 = wt.view(1, F, d)

    def a_path():
        return ops.swiglu_bwd(mm(dy, wt.t()), gu)

    def b_path():
        return gm.grouped_dx_swiglu(dy, w3, offs, gu)

    ra, rb = a_path().float(), b_path().float()
    da = mm(dy, wt.t())
    rel = float((ra - rb).abs().max() / ra.abs().max())
    flop = 2.0 * T * d * F
    res = {"shape": [T, d, F],
           "A_hipblaslt_plus_swiglu_us": timeit(a_path), "B_mfma_fused_us": timeit(b_path),
           "hipblaslt_gemm_us": timeit(lambda: mm(dy, wt.t())),
           "mfma_grouped_g1_gemm_us": timeit(lambda: gm.grouped_mm(dy, w3, offs)),
           "swiglu_bwd_us": timeit(lambda: ops.swiglu_bwd(da, gu)),
           "max_rel_diff_A_vs_B": rel}
    res["hipblaslt_pflops"] = flop / res["hipblaslt_gemm_us"] / 1e9
    res["mfma_pflops"] = flop / res["mfma_grouped_g1_gemm_us"] / 1e9
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
