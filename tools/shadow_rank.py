#!/usr/bin/env python3
"""Shadow-rank run: rank r of a world-W ZeRO job, alone on ONE MI355X.

The engine is built with ``parallel.comm.ShadowComm(W, r)``: it allocates exactly what rank r of
the real job allocates (1/W shards of the fp32 master / m / v / gradients and bf16 parameters,
full-size all-gather / reduce-scatter / all-to-all buffers, the ZeRO-3 residency plan sized for
W ranks) and every collective becomes a local device copy of the true size. Reported:

* ``peak_GiB`` -- torch.cuda.max_memory_allocated over the whole run, and the planner's prediction
  (``parallel/planner.py``) for the same configuration;
* per-rank step time -- compute + local memory traffic only: xGMI transfer time is NOT included,
  so this is never a headline or scaling number.

    python tools/shadow_rank.py --model llama3-70b --world 8 --ga 2 --ckpt --out gpurun_out/shadow_70b.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _knob(v: str):
    return v if v in ("hbm", "auto") else float(v)


def _comms(eng):
    seen = {}
    for c in [eng.comm, getattr(eng, "gather_comm", None), getattr(eng, "ep_comm", None),
              getattr(eng, "edp_comm", None)] + [x for g in eng.groups for x in (g.comm, getattr(g, "gcomm", None))]:
        if c is not None:
            seen[id(c)] = c
    return list(seen.values())


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--zero", type=int, default=3)
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--mbs", type=int, default=1)
    ap.add_argument("--ga", type=int, default=2, help="micro-batches per step in this run (the preset's GA only "
                    "changes how often the optimizer runs, not the per-rank memory)")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--ckpt", action="store_true", help="activation checkpointing")
    ap.add_argument("--ep", type=int, default=1, help="expert-parallel size (Mixtral)")
    ap.add_argument("--n-layers", type=int, default=0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--async-comm", action="store_true",
                    help="collectives on per-communicator HIP streams, ordered like RCCL's (ShadowComm async_mode)")
    ap.add_argument("--link-gbps", type=float, default=0.0,
                    help="async comm: hold each collective's stream for its ring time at this xGMI bus bandwidth")
    ap.add_argument("--a2a-gbps", type=float, default=0.0, help="all-to-all bandwidth of the link model (default: link)")
    ap.add_argument("--live-params", default="hbm", help="stage3_max_live_parameters: 'hbm' or a number (1e9: reference)")
    ap.add_argument("--reuse-distance", default="hbm", help="stage3_max_reuse_distance: 'hbm' or a number")
    ap.add_argument("--local-grads", default="hbm", help="'hbm', 'on' or 'off' (off: reduce-scatter every micro-batch)")
    ap.add_argument("--engine-kw", default="", help="more EngineConfig fields, 'name=value,...' (numbers parsed)")
    a = ap.parse_args(argv)

    import torch

    from distributed_llm_training_gpu_manager_amd import _native
    from distributed_llm_training_gpu_manager_amd.models import get_config
    from distributed_llm_training_gpu_manager_amd.parallel.comm import ShadowComm
    from distributed_llm_training_gpu_manager_amd.parallel.planner import GiB, plan_rank
    from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    _native.hip_ops()
    mcfg = get_config(a.model, **({"n_layers": a.n_layers} if a.n_layers else {}))
    ecfg = EngineConfig(zero_stage=a.zero, micro_batch_size=a.mbs, seq_len=a.seq, grad_accum=a.ga, lr=3e-5,
                        warmup_steps=100, total_steps=10000, grad_clip=1.0, activation_checkpointing=a.ckpt,
                        max_live_parameters=_knob(a.live_params), max_reuse_distance=_knob(a.reuse_distance),
                        local_grad_accum={"on": True, "off": False}.get(a.local_grads, a.local_grads),
                        expert_parallel_size=a.ep)
    for kv in filter(None, a.engine_kw.split(",")):
        k, v = kv.split("=", 1)
        try:
            v = float(v) if "." in v or "e" in v else int(v)
        except ValueError:
            pass
        setattr(ecfg, k, v)
    t0 = time.time()
    comm = ShadowComm(a.world, a.rank, async_mode=a.async_comm or a.link_gbps > 0, link_gbps=a.link_gbps,
                      a2a_gbps=a.a2a_gbps)
    eng = ZeroEngine(mcfg, ecfg, dev, comm)
    torch.cuda.synchronize()
    init_s = time.time() - t0
    print(f"[shadow] {mcfg.name} rank {a.rank}/{a.world}: engine built in {init_s:.1f}s, "
          f"{torch.cuda.memory_allocated() / GiB:.1f} GiB allocated", flush=True)
    gen = torch.Generator(device=dev)
    gen.manual_seed(7 + a.rank)
    total = a.warmup + a.steps
    data = []
    for _ in range(total):
        mb = []
        for _ in range(a.ga):
            toks = torch.randint(0, mcfg.vocab_size, (a.mbs, a.seq + 1), device=dev, generator=gen)
            mb.append((toks[:, :-1].contiguous(), toks[:, 1:].contiguous()))
        data.append(mb)
    times = []
    for i in range(total):
        torch.cuda.synchronize()
        t = time.perf_counter()
        m = eng.train_step(data[i])
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t)
        print(f"[shadow] step {i + 1}/{total}: {times[-1]:.2f}s loss={float(m['loss']):.3f} "
              f"peak={torch.cuda.max_memory_allocated() / GiB:.1f} GiB", flush=True)
    timed = times[a.warmup:] or times
    plan = plan_rank(mcfg, world=a.world, zero_stage=a.zero, micro_batch=a.mbs, seq_len=a.seq, grad_accum=a.ga,
                     activation_checkpointing=a.ckpt, ep_size=a.ep,
                     hbm_bytes=torch.cuda.get_device_properties(dev).total_memory)
    rep = eng.memory_report()
    peak = torch.cuda.max_memory_allocated() / GiB
    hbm = torch.cuda.get_device_properties(dev).total_memory / GiB
    out = {
        "what": "shadow rank: one rank of a world-W job alone on one MI355X (collectives = local copies of the "
                "true size); per-rank memory + compute time, NOT a throughput/scaling number",
        "model": mcfg.name, "n_layers": mcfg.n_layers, "params": eng.num_params(), "world": a.world,
        "rank": a.rank, "zero_stage": a.zero, "ep_size": eng.ep_size, "seq_len": a.seq, "micro_batch": a.mbs,
        "grad_accum_in_run": a.ga, "activation_checkpointing": a.ckpt,
        "peak_GiB": round(peak, 2), "hbm_GiB": round(hbm, 2), "headroom": round(1 - peak / hbm, 4),
        "planned_GiB": round(plan.total / GiB, 2), "planned_parts_GiB": plan.summary()["parts_GiB"],
        "engine_mem_GiB": {k: round(v, 2) for k, v in rep.items()},
        "zero3_resident_groups": len(eng.live_plan.resident_groups),
        "zero3_allgathers_per_step": eng.live_plan.gathers_per_step(a.ga),
        "step_s": [round(x, 3) for x in times], "per_micro_batch_s": round(sum(timed) / len(timed) / a.ga, 3),
        "tokens_per_s_per_rank_compute_only": round(a.mbs * a.seq * a.ga * len(timed) / sum(timed), 1),
        "init_s": round(init_s, 1),
        "comm": "async (per-communicator HIP streams, RCCL ordering)" if (a.async_comm or a.link_gbps > 0)
        else "sync (compute stream)",
        "async_collectives_issued": sum(getattr(c, "issued", 0) for c in _comms(eng)),
        "link_model": {"link_gbps": a.link_gbps, "a2a_gbps": a.a2a_gbps or a.link_gbps,
                       "modelled_link_s_total": round(sum(getattr(c, "modelled_s", 0.0) for c in _comms(eng)), 3),
                       "steps_in_run": total} if a.link_gbps > 0 else None,
        "knobs": {"stage3_max_live_parameters": a.live_params, "stage3_max_reuse_distance": a.reuse_distance,
                  "local_grads": eng.local_grads, "gathers_per_step": eng.live_plan.gathers_per_step(a.ga)},
    }
    print(json.dumps(out), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
