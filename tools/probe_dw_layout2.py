"""dW GEMM layouts with the HIP transpose: GEMM-only time per operand layout + transpose cost."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributed_llm_training_gpu_manager_amd.ops.gemm import transpose  # noqa: E402


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
acc = lambda g, a, b: torch.addmm(g, a, b, beta=1.0, out_dtype=torch.float32, out=g)  # noqa: E731
for name, (N, K) in shapes.items():
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    g = torch.zeros(N, K, device="cuda", dtype=torch.float32)
    dyT, xT = transpose(dy), transpose(x)
    assert torch.equal(dyT, dy.t().contiguous()) and torch.equal(xT, x.t().contiguous())
    fl = 2.0 * T * N * K
    r = {
        "NN": bench(lambda: acc(g, dy.t(), x)),
        "TN": bench(lambda: acc(g, dyT, xT.t())),
        "dyT_x": bench(lambda: acc(g, dyT, x)),
        "dy_xT": bench(lambda: acc(g, dy.t(), xT.t())),
    }
    tdy = bench(lambda: transpose(dy, dyT))
    tx = bench(lambda: transpose(x, xT))
    cost = {"NN": r["NN"], "TN": r["TN"] + tdy + tx, "dyT_x": r["dyT_x"] + tdy, "dy_xT": r["dy_xT"] + tx}
    best = min(cost, key=cost.get)
    print(f"{name:10s} gemm " + " ".join(f"{k}={v:.3f}({fl / v / 1e9:.0f}TF)" for k, v in r.items()) +
          f" | transpose dy {tdy:.3f}ms ({2 * dy.numel() * 2 / tdy / 1e9:.0f} GB/s) x {tx:.3f}ms"
          f" | total " + " ".join(f"{k}={v:.3f}" for k, v in cost.items()) + f" -> {best}", flush=True)
    del dy, x, g, dyT, xT
