"""Timing + bit-exactness probe of the hand MFMA GEMM on the Mixtral-8x7B expert shapes (one process per build /
schedule; prints one JSON line). Shapes: grouped-M forward w13 (N 28672, K 4096) and w2 (N 4096, K 14336), the
input-gradient GEMMs (N 4096, K 28672 / N 14336, K 4096), the K-major segmented dW over 4 micro-batches, and the
dense 8192 x 28672 x 4096 forward layout. Random bf16 operands, uneven expert counts like the random-init router."""
import hashlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_llm_training_gpu_manager_amd.ops import gemm_mfma as gm  # noqa: E402
from distributed_llm_training_gpu_manager_amd.ops.gemm import transpose  # noqa: E402
from distributed_llm_training_gpu_manager_amd.ops.moe import pad_plan  # noqa: E402


def _digest(t: torch.Tensor) -> str:
    return hashlib.sha1(t.contiguous().view(torch.uint8).cpu().numpy().tobytes()).hexdigest()[:12]


def _time(fn, iters):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(iters):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / iters


def main():
    dev = "cuda"
    torch.manual_seed(0)
    counts = [1320, 870, 1105, 940, 1010, 1190, 760, 997]
    E, d, F = 8, 4096, 14336
    R = sum(counts)
    offs = torch.zeros(E + 1, dtype=torch.int32)
    offs[1:] = torch.tensor(counts).cumsum(0)
    offs = offs.to(dev)
    res = {"sched": os.environ.get("DLGM_GEMM_SCHED", "0")}
    iters = int(os.environ.get("ITERS", "10"))

    def grouped(name, K, N, transpose_w):
        x = torch.randn(R, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(E, N, K, device=dev) * 0.02).to(torch.bfloat16) if transpose_w else \
            (torch.randn(E, K, N, device=dev) * 0.02).to(torch.bfloat16)
        out = torch.empty(R, N, device=dev, dtype=torch.bfloat16)
        ms = _time(lambda: gm.grouped_mm(x, w, offs, transpose_w=transpose_w, out=out), iters)
        res[name] = {"ms": round(ms, 4), "TFs": round(2.0 * R * K * N / ms / 1e9, 1), "sha": _digest(out)}

    grouped("fwd_w13", d, 2 * F, True)        # x @ w13^T: w [E, 28672, 4096]
    grouped("fwd_w2", F, d, True)             # a @ w2^T: w [E, 4096, 14336]
    grouped("dx_w13", 2 * F, d, True)         # dgu @ w13 through the engine's [E, in, out] W^T cache
    grouped("da_w2", d, F, True)              # dy @ w2 through the cache ([E, 14336, 4096])
    grouped("dx_w13_mn", 2 * F, d, False)     # the same two straight from the [E, out, in] weights (MN-contiguous B)
    grouped("da_w2_mn", d, F, False)

    src, poff = pad_plan(offs, R, 64)
    for name, M in (("dw_w13", 2 * F), ("dw_w2", d)):
        N = F if M == d else d
        a_t = [transpose(torch.randn(R, M, device=dev).to(torch.bfloat16), rows=src) for _ in range(4)]
        b_t = [transpose(torch.randn(R, N, device=dev).to(torch.bfloat16), rows=src) for _ in range(4)]
        offs_s = torch.stack([poff] * 4)
        out = torch.zeros(E, M, N, device=dev)
        ms = _time(lambda: gm.grouped_wgrad_segments(out, a_t, b_t, offs_s, kmajor=True), max(2, iters // 3))
        res[name] = {"ms": round(ms, 4), "TFs": round(2.0 * 4 * R * M * N / ms / 1e9, 1), "sha": _digest(out)}
        del a_t, b_t, out

    # the engine's dW path: the step's 4 micro-batches re-laid into ONE K-major operand (transpose_multi), one
    # grouped-K launch per weight (mode 2)
    from distributed_llm_training_gpu_manager_amd.ops.gemm import transpose_multi
    from distributed_llm_training_gpu_manager_amd.ops.moe import pad_plan_multi
    offs_m = torch.stack([offs] * 4)
    src_m, poff_m = pad_plan_multi(offs_m, 4 * R)
    for name, M in (("dw1_w13", 2 * F), ("dw1_w2", d)):
        N = F if M == d else d
        at = transpose_multi([torch.randn(R, M, device=dev).to(torch.bfloat16) for _ in range(4)], src_m)
        bt = transpose_multi([torch.randn(R, N, device=dev).to(torch.bfloat16) for _ in range(4)], src_m)
        out = torch.zeros(E, M, N, device=dev)
        ms = _time(lambda: gm.grouped_wgrad(out, at, bt, poff_m, acc=True, kmajor=True), max(2, iters // 3))
        res[name] = {"ms": round(ms, 4), "TFs": round(2.0 * 4 * R * M * N / ms / 1e9, 1), "sha": _digest(out)}
        del at, bt, out

    a = torch.randn(R, d, device=dev).to(torch.bfloat16)
    b = torch.randn(2 * F, d, device=dev).to(torch.bfloat16)
    o = torch.empty(R, 2 * F, device=dev, dtype=torch.bfloat16)
    ms = _time(lambda: gm.mfma_mm(o, a, b.t()), iters)
    res["dense_fwd"] = {"ms": round(ms, 4), "TFs": round(2.0 * R * d * 2 * F / ms / 1e9, 1), "sha": _digest(o)}
    del a, b, o
    # the MoE dW re-layout (4 micro-batch sources, expert-aligned columns) and a plain expert W^T transpose
    from distributed_llm_training_gpu_manager_amd.ops.gemm import transpose_multi
    from distributed_llm_training_gpu_manager_amd.ops.moe import pad_plan_multi
    offs_m = torch.stack([offs] * 4)
    src_m, _ = pad_plan_multi(offs_m, 4 * R)
    for name, C in (("tmulti_dgu", 2 * F), ("tmulti_x", d)):
        xs = [torch.randn(R, C, device=dev).to(torch.bfloat16) for _ in range(4)]
        ms = _time(lambda: transpose_multi(xs, src_m), iters)
        y = transpose_multi(xs, src_m)
        res[name] = {"ms": round(ms, 4), "TBs": round(2.0 * 2 * y.numel() / ms / 1e9, 2), "sha": _digest(y)}
        del xs, y
    big = torch.randn(4 * R, 2 * F, device=dev).to(torch.bfloat16)  # tmulti_dgu's shape without the remap
    ms = _time(lambda: transpose(big), iters)
    res["t_big"] = {"ms": round(ms, 4), "TBs": round(2.0 * 2 * big.numel() / ms / 1e9, 2)}
    ident = torch.arange(big.shape[0], dtype=torch.int32, device=dev)  # the remap path with the identity map
    ms = _time(lambda: transpose(big, rows=ident), iters)
    res["t_big_remap_id"] = {"ms": round(ms, 4), "TBs": round(2.0 * 2 * big.numel() / ms / 1e9, 2)}
    perm = src_m.clone()
    perm[perm >= 0] = torch.arange(int((perm >= 0).sum()), dtype=torch.int32, device=dev)  # the expert plan's
    ms = _time(lambda: transpose(big, rows=perm[:big.shape[0]]), iters)                   # padding, one source
    res["t_big_remap_pad"] = {"ms": round(ms, 4), "TBs": round(2.0 * 2 * big.numel() / ms / 1e9, 2)}
    P = src_m.shape[0]
    big2 = torch.randn(P, 2 * F, device=dev).to(torch.bfloat16)  # plain, with tmulti_dgu's padded row count
    ms = _time(lambda: transpose(big2), iters)
    res["t_big_P"] = {"ms": round(ms, 4), "TBs": round(2.0 * 2 * big2.numel() / ms / 1e9, 2), "P": P}
    del big2
    del big
    w = torch.randn(2 * F, d, device=dev).to(torch.bfloat16)
    wt = torch.empty(d, 2 * F, device=dev, dtype=torch.bfloat16)
    ms = _time(lambda: transpose(w, out=wt), iters)
    res["t_w13"] = {"ms": round(ms, 4), "TBs": round(2.0 * 2 * w.numel() / ms / 1e9, 2), "sha": _digest(wt)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
