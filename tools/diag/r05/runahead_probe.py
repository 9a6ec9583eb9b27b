"""Round-5 flake probe, stage 6: does the result depend on how far the host runs ahead of the GPU? The failing
engine's side work was serialised behind the shadow comm's spin kernels (its streams were the side streams' HIP
streams), i.e. its GPU fell further behind the host than in the later engines. Here the GPU is held back on
purpose: before every train_step (and optionally every micro-batch) a long spin kernel is queued on the compute
stream, so the host queues a whole step of kernels -- and every host-side argument / staging buffer of the libraries
it calls -- before the GPU starts on them. Compared bit for bit with the same engine without the spin."""
import json
import os
import sys

import torch

sys.path.insert(0, ".")
from distributed_llm_training_gpu_manager_amd.models import get_config  # noqa: E402
from distributed_llm_training_gpu_manager_amd.parallel.comm import ShadowComm  # noqa: E402
from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine  # noqa: E402

dev = torch.device("cuda", 0)


def run(model, spin, per_micro=False, blas=None, world=4):
    if blas:
        torch.backends.cuda.preferred_blas_library(blas)
    mc = get_config(model)
    ec = EngineConfig(micro_batch_size=2, seq_len=64, grad_accum=2, lr=1e-3, scheduler="constant", grad_clip=1.0,
                      zero_stage=3, expert_parallel_size=4 if (model == "mixtral-tiny" and world == 4) else 1,
                      local_grad_accum=False, optimizer_overlap=False)
    comm = ShadowComm(world, 0, async_mode=True, delay_cycles=200_000) if world > 1 else None
    eng = ZeroEngine(mc, ec, dev, comm)
    if per_micro and spin:
        orig = eng.micro_step

        def ms(*a, **k):
            torch.cuda._sleep(spin)
            return orig(*a, **k)
        eng.micro_step = ms
    g = torch.Generator().manual_seed(3)
    for _ in range(3):
        mbs = []
        for _ in range(2):
            t = torch.randint(0, mc.vocab_size, (2, 65), generator=g).to(dev)
            mbs.append((t[:, :-1].contiguous(), t[:, 1:].contiguous()))
        if spin and not per_micro:
            torch.cuda._sleep(spin)
        eng.train_step(mbs)
    torch.cuda.synchronize()
    if blas:
        torch.backends.cuda.preferred_blas_library("cublaslt")
    return {k: getattr(eng, k).detach().cpu().clone() for k in ("master", "grad_shard")}


out = {}
for model, world in (("mixtral-tiny", 4), ("llama-tiny", 4), ("mixtral-tiny", 1)):
    ref = run(model, 0, world=world)
    for name, kw in (("spin_step", dict(spin=1_500_000_000)), ("spin_micro", dict(spin=600_000_000, per_micro=True)),
                     ("no_spin_repeat", dict(spin=0))):
        r = run(model, world=world, **kw)
        out[f"{model}_w{world}_{name}"] = {k: (bool(torch.equal(r[k], ref[k])),
                                               float((r[k].float() - ref[k].float()).abs().max())) for k in ref}
        print(f"{model}_w{world}_{name}", out[f"{model}_w{world}_{name}"], flush=True)
os.makedirs("gpurun_out/digest", exist_ok=True)
with open("gpurun_out/digest/runahead_probe.json", "w") as f:
    json.dump(out, f, indent=1)
