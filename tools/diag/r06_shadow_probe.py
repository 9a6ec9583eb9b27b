#!/usr/bin/env python3
"""Round 6: per-step loss / grad-norm / master checksums of the synchronous and asynchronous shadow runs of TARGET
after the interleaved case sequence of r06_shadow_stress.py -- in which step, and before or after the optimizer, the
asynchronous run first differs. EMPTY_CACHE=1: gc + empty_cache before every run (allocator state reset)."""
import gc
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
import torch  # noqa: E402
import test_shadow_async_gpu as T  # noqa: E402
from distributed_llm_training_gpu_manager_amd.models import get_config  # noqa: E402
from distributed_llm_training_gpu_manager_amd.parallel.comm import ShadowComm  # noqa: E402
from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine  # noqa: E402


def run(case, async_mode, steps=3, ga=2):
    if os.environ.get("EMPTY_CACHE") == "1":
        gc.collect()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    dev = torch.device("cuda", 0)
    mc = get_config("llama-tiny")
    ec = EngineConfig(micro_batch_size=2, seq_len=64, grad_accum=ga, lr=1e-3, scheduler="constant", grad_clip=1.0)
    for k, v in T.CASES[case].items():
        setattr(ec, k, v)
    comm = ShadowComm(4, 0, async_mode=async_mode, delay_cycles=200_000 if async_mode else 0)
    eng = ZeroEngine(mc, ec, dev, comm)
    g = torch.Generator().manual_seed(3)
    rec = []
    for _ in range(steps):
        mbs = []
        for _ in range(ga):
            t = torch.randint(0, mc.vocab_size, (2, 65), generator=g).to(dev)
            mbs.append((t[:, :-1].contiguous(), t[:, 1:].contiguous()))
        m = eng.train_step(mbs)
        torch.cuda.synchronize()
        rec.append({"loss": float(m["loss"]), "gnorm": float(m["grad_norm"]),
                    "master": float(eng.master.double().sum()), "grad": float(eng.grad_shard.double().abs().sum()),
                    "p16": float(eng.p16_shard.double().sum())})
    return rec


def main():
    target = os.environ.get("TARGET", "zero3_offload_param")
    reps = int(os.environ.get("REPS", "4"))
    cases = sorted(T.CASES)
    ref = run(target, False)
    print(json.dumps({"ref": ref}), flush=True)
    for c in cases:
        if c != target:
            run(c, False)
    shown = 0
    for i in range(reps):
        for c in cases:
            if c != target:
                run(c, True)
                continue
            got = run(target, True)
            if got != ref:
                first = next((s, k) for s in range(len(ref)) for k in ref[s] if ref[s][k] != got[s][k])
                print(json.dumps({"rep": i, "first_diff_step_key": first, "got": got}), flush=True)
                shown += 1
            else:
                print(json.dumps({"rep": i, "equal": True}), flush=True)


if __name__ == "__main__":
    main()
