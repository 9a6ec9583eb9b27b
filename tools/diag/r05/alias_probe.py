"""Round-5 flake probe, stage 5: reproduce the first-engine mismatch on purpose in a fresh process. The failing engine
was the one whose shadow-comm HIP streams happened to be the engine's own side streams (torch's 32-stream pool wraps
round-robin): gather_comm == the W^T-cache stream, ep_comm == the MoE dW re-layout stream. Here those aliases are
forced one at a time on the Mixtral-tiny EP-4 ZeRO-3 engine of the round-4 test; each run is compared bit for bit
with the same engine on distinct streams, three steps."""
import json
import os
import sys

import torch

sys.path.insert(0, ".")
from distributed_llm_training_gpu_manager_amd.models import get_config  # noqa: E402
from distributed_llm_training_gpu_manager_amd.parallel.comm import ShadowComm  # noqa: E402
from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine  # noqa: E402
from distributed_llm_training_gpu_manager_amd.utils.streams import side_stream  # noqa: E402

dev = torch.device("cuda", 0)


def run(alias, model="mixtral-tiny", **kw):
    mc = get_config(model)
    ec = EngineConfig(micro_batch_size=2, seq_len=64, grad_accum=2, lr=1e-3, scheduler="constant", grad_clip=1.0,
                      zero_stage=3, expert_parallel_size=4 if model == "mixtral-tiny" else 1, local_grad_accum=False,
                      optimizer_overlap=False, **kw)
    eng = ZeroEngine(mc, ec, dev, ShadowComm(4, 0, async_mode=True, delay_cycles=200_000))
    pairs = {"gather=tcache": ("gather_comm", "tcache"), "ep=moe_dw": ("ep_comm", "moe_dw"),
             "comm=tcache": ("comm", "tcache"), "comm=moe_dw": ("comm", "moe_dw"),
             "ep=tcache": ("ep_comm", "tcache"), "gather=moe_dw": ("gather_comm", "moe_dw")}
    for a in alias:
        if a not in pairs:
            continue
        attr, side = pairs[a]
        c = getattr(eng, attr, None)
        if c is not None:
            c._stream = side_stream(dev, side)
    if "comm=gather" in alias:
        eng.gather_comm._stream = eng.comm._stream = torch.cuda.Stream(dev)
    g = torch.Generator().manual_seed(3)
    for _ in range(3):
        mbs = []
        for _ in range(2):
            t = torch.randint(0, mc.vocab_size, (2, 65), generator=g).to(dev)
            mbs.append((t[:, :-1].contiguous(), t[:, 1:].contiguous()))
        eng.train_step(mbs)
    torch.cuda.synchronize()
    return {k: getattr(eng, k).detach().cpu().clone() for k in ("master", "grad_shard")}


out = {}
model = os.environ.get("MODEL", "mixtral-tiny")
ref = run([], model)
ref2 = run([], model)
out["ref_repeat_equal"] = all(torch.equal(ref[k], ref2[k]) for k in ref)
for alias in (["gather=tcache"], ["ep=moe_dw"], ["gather=tcache", "ep=moe_dw"], ["comm=tcache"], ["comm=moe_dw"],
              ["ep=tcache"], ["gather=moe_dw"], ["comm=gather"]):
    res = [run(alias, model) for _ in range(2)]
    out["+".join(alias)] = [{k: (bool(torch.equal(r[k], ref[k])),
                                 float((r[k].float() - ref[k].float()).abs().max())) for k in ref} for r in res]
    print("+".join(alias), out["+".join(alias)], flush=True)
os.makedirs("gpurun_out/digest", exist_ok=True)
with open(f"gpurun_out/digest/alias_probe_{model}.json", "w") as f:
    json.dump(out, f, indent=1)
print(json.dumps(out)[:3000])
