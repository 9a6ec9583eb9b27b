"""PMC / timing probe: the grouped-M MFMA GEMM at the Mixtral-8x7B w13 shape (8192 routed rows, uneven experts)
against the dense kernel on the same 8192 x 4096 x 28672 problem (one weight). Random bf16 operands."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_llm_training_gpu_manager_amd.ops import gemm_mfma as gm  # noqa: E402


def main():
    dev = "cuda"
    counts = [1320, 870, 1105, 940, 1010, 1190, 760, 997]  # 8192 rows, imbalance like the random-init router
    E, d, N = 8, 4096, 28672
    offs = torch.zeros(E + 1, dtype=torch.int32)
    offs[1:] = torch.tensor(counts).cumsum(0)
    offs = offs.to(dev)
    x = torch.randn(sum(counts), d, device=dev).to(torch.bfloat16)
    w = (torch.randn(E, N, d, device=dev) * 0.02).to(torch.bfloat16)
    out = torch.empty(sum(counts), N, device=dev, dtype=torch.bfloat16)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    for _ in range(2):
        gm.grouped_mm(x, w, offs, out=out)
        gm.mfma_mm(out, x, w[0].t())
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(5):
        gm.grouped_mm(x, w, offs, out=out)
    ev[1].record()
    for _ in range(5):
        gm.mfma_mm(out, x, w[0].t())
    ev[2].record()
    torch.cuda.synchronize()
    f = 2.0 * sum(counts) * d * N
    tg, td = ev[0].elapsed_time(ev[1]) / 5, ev[1].elapsed_time(ev[2]) / 5
    print(f"w13-like N {N} K {d}: grouped {tg:.3f} ms {f / tg / 1e9:.0f} TF/s | dense {td:.3f} ms {f / td / 1e9:.0f} TF/s")
    # the narrow grouped GEMMs of the step: N = 4096 (16 column tiles), K = 28672 (dX of w13) and K = 14336 (w2)
    for K2 in (28672, 14336):
        x2 = torch.randn(sum(counts), K2, device=dev).to(torch.bfloat16)
        w2 = (torch.randn(E, d, K2, device=dev) * 0.02).to(torch.bfloat16)
        o2 = torch.empty(sum(counts), d, device=dev, dtype=torch.bfloat16)
        gm.grouped_mm(x2, w2, offs, out=o2)
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(5):
            gm.grouped_mm(x2, w2, offs, out=o2)
        ev[1].record()
        torch.cuda.synchronize()
        t2 = ev[0].elapsed_time(ev[1]) / 5
        f2 = 2.0 * sum(counts) * d * K2
        print(f"narrow N {d} K {K2}: grouped {t2:.3f} ms {f2 / t2 / 1e9:.0f} TF/s")


def seg_dw():
    """K-major segmented grouped dW (4 micro-batches x 8 experts, Mixtral w13 dW [8, 28672, 4096]) against the dense
    kernel on one expert-sized K-major problem (x 8)."""
    from distributed_llm_training_gpu_manager_amd.ops.gemm import transpose
    from distributed_llm_training_gpu_manager_amd.ops.moe import pad_plan
    dev = "cuda"
    counts = [1320, 870, 1105, 940, 1010, 1190, 760, 997]
    E, M, N = 8, 28672, 4096
    R = sum(counts)
    offs = torch.zeros(E + 1, dtype=torch.int32)
    offs[1:] = torch.tensor(counts).cumsum(0)
    src, poff = pad_plan(offs.to(dev), R, 64)
    a_t, b_t = [], []
    for _ in range(4):
        a_t.append(transpose(torch.randn(R, M, device=dev).to(torch.bfloat16), rows=src))
        b_t.append(transpose(torch.randn(R, N, device=dev).to(torch.bfloat16), rows=src))
    offs_s = torch.stack([poff] * 4)
    out = torch.zeros(E, M, N, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    gm.grouped_wgrad_segments(out, a_t, b_t, offs_s, kmajor=True)
    K1 = 4 * 1024
    a1 = torch.randn(M, K1, device=dev).to(torch.bfloat16)
    b1 = torch.randn(N, K1, device=dev).to(torch.bfloat16)
    o1 = torch.zeros(M, N, device=dev)
    gm.mfma_mm(o1, a1, b1.t())
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(3):
        gm.grouped_wgrad_segments(out, a_t, b_t, offs_s, kmajor=True)
    ev[1].record()
    for _ in range(3):
        for _e in range(E):
            gm.mfma_mm(o1, a1, b1.t())
    ev[2].record()
    torch.cuda.synchronize()
    ts, td = ev[0].elapsed_time(ev[1]) / 3, ev[1].elapsed_time(ev[2]) / 3
    f = 2.0 * 4 * R * M * N
    fd = 2.0 * E * K1 * M * N
    print(f"seg dW kmajor {ts:.3f} ms {f / ts / 1e9:.0f} TF/s | dense x8 (K {K1}) {td:.3f} ms {fd / td / 1e9:.0f} TF/s")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "seg":
        seg_dw()
        sys.exit(0)
    main()
