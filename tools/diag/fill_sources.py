"""Which host ops launch the fp32 fill kernels in a Llama-3-8B step (diagnostic; 4 layers, GA 2, 1 GPU).

Runs one profiled engine step under torch.profiler and, for every GPU kernel whose name contains
"Fill" / copies / elementwise, prints the chain of CPU ops that launched it with the kernel's total time."""
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from distributed_llm_training_gpu_manager_amd.models import get_config  # noqa: E402
from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine  # noqa: E402


PATTERNS = ("Fill", "copyBuffer", "Copy", "CatArray", "elementwise", "transpose", "reduce")


def main():
    dev = torch.device("cuda")
    model = sys.argv[1] if len(sys.argv) > 1 else "llama3-8b"
    mc = get_config(model, n_layers=2 if model != "llama3-8b" else 4)
    seq = 8192 if model == "llama3-8b" else 4096
    ec = EngineConfig(zero_stage=3, micro_batch_size=1, seq_len=seq, grad_accum=2, lr=1e-4)
    eng = ZeroEngine(mc, ec, dev)
    mbs = [(torch.randint(0, mc.vocab_size, (1, seq), device=dev),) * 2 for _ in range(2)]
    for _ in range(2):
        eng.train_step(mbs)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        eng.train_step(mbs)
        torch.cuda.synchronize()
    agg = collections.defaultdict(lambda: [0, 0.0])
    for cpu in prof.events():
        for k in getattr(cpu, "kernels", []):
            tag = next((t for t in PATTERNS if t in k.name), None)
            if tag is None:
                continue
            chain, q = [], cpu
            while q is not None:
                chain.append(q.name)
                q = q.cpu_parent
            a = agg[tag + ": " + " <- ".join(chain[:7])]
            a[0] += 1
            a[1] += k.duration
    for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{n:5d} {us / 1000:9.2f} ms  {k}")


if __name__ == "__main__":
    main()
