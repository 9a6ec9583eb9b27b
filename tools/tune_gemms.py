"""Tune the Llama-3 GEMM shapes with PyTorch TunableOp (hipBLASLt + rocBLAS solution search).

WARNING: the exhaustive search launches every candidate solution; on ROCm 7.0 / gfx950 one
candidate for the [8192 x 28672] x [28672 x 4096] input-gradient GEMM faulted the GPU
("unspecified launch failure"). Do not run this on shared machines; the framework does not
depend on tuned files (utils/gemm_tuning.py loads them only if present).

Writes the winning solutions to ``distributed_llm_training_gpu_manager_amd/tuned/`` (loaded by
``utils.gemm_tuning.enable_tuned_gemms``) and prints default-vs-tuned times per shape.

    python tools/tune_gemms.py --model llama3-8b --tokens 8192
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_llm_training_gpu_manager_amd.models import get_config  # noqa: E402


def shapes(cfg, T):
    ws = {"wqkv": (cfg.qkv_dim, cfg.d_model), "wo": (cfg.d_model, cfg.n_heads * cfg.head_dim),
          "w_gate_up": (2 * cfg.ffn_dim, cfg.d_model), "w_down": (cfg.d_model, cfg.ffn_dim),
          "lm_head": (cfg.vocab_size, cfg.d_model)}
    return ws


def _write(fname: str) -> None:
    """TunableOp results file: validator lines, then op,params,solution,ms lines."""
    tun = torch.cuda.tunable
    lines = [f"Validator,{k},{v}" for k, v in tun.get_validators()]
    lines += [",".join(str(x) for x in r) for r in tun.get_results()]
    tmp = fname + ".tmp"
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, fname)


def bench(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--out", default=None)
    ap.add_argument("--max-ms", type=int, default=30)
    ap.add_argument("--max-iters", type=int, default=20)
    a = ap.parse_args()
    cfg = get_config(a.model)
    T = a.tokens
    dev = "cuda"
    out_dir = a.out or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "distributed_llm_training_gpu_manager_amd", "tuned")
    os.makedirs(out_dir, exist_ok=True)
    cases = []
    for name, (N, K) in shapes(cfg, T).items():
        x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        dy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * T * N * K
        # the fp32-output (aten mm.dtype_out) weight-gradient GEMMs are not covered by TunableOp
        cases += [
            (name + ".fwd", fl, lambda x=x, w=w: torch.mm(x, w.t())),
            (name + ".dx", fl, lambda dy=dy, w=w: torch.mm(dy, w)),
        ]
    res = {}
    for n, fl, fn in cases:
        res[n] = {"default_ms": bench(fn)}
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(a.max_ms)
    tun.set_max_tuning_iterations(a.max_iters)
    fname = os.path.join(out_dir, f"tunableop_{a.model}_T{T}.csv")
    tun.set_filename(fname)
    for n, fl, fn in cases:
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        res[n]["tune_s"] = time.perf_counter() - t0
        print(f"tuned {n} in {res[n]['tune_s']:.1f}s", flush=True)
        _write(fname)  # keep what is tuned so far (TunableOp itself only writes at process exit)
    tun.tuning_enable(False)
    for n, fl, fn in cases:
        res[n]["tuned_ms"] = bench(fn)
        res[n]["default_TF"] = fl / res[n]["default_ms"] / 1e9
        res[n]["tuned_TF"] = fl / res[n]["tuned_ms"] / 1e9
        print(f"{n:22s} default {res[n]['default_ms']:7.3f} ms {res[n]['default_TF']:7.1f} TF | "
              f"tuned {res[n]['tuned_ms']:7.3f} ms {res[n]['tuned_TF']:7.1f} TF", flush=True)
    print(json.dumps({"file": fname, "results": res}))


if __name__ == "__main__":
    main()
