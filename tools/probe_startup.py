#!/usr/bin/env python3
"""Where does the first training step's extra time go (70B rank-scale MTTR, first step 16.9 s
vs a few seconds steady)? Rank `--shadow-rank` of a `--shadow-world` ZeRO-3 job alone on this GPU (the drill's
setup): engine construction, then N steps, each unit's forward / backward bracketed by a device sync and timed,
plus the allocator's reserved bytes and the number of hipMalloc-backed segments after each step.

  python tools/probe_startup.py --model llama3-70b --seq 8192 --steps 3 [--warm ...]
prints one JSON line; --out writes it too."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--shadow-world", type=int, default=8)
    ap.add_argument("--ckpt", type=int, default=1, help="activation checkpointing")
    ap.add_argument("--n-layers", type=int, default=0)
    ap.add_argument("--warm", default="none", help="none | engine (ZeroEngine.warm_up before step 1)")
    ap.add_argument("--per-unit", type=int, default=1, help="sync + time every unit (changes overlap)")
    ap.add_argument("--ckpt-tier", dest="ckpt_tier", default="none", help="none | shm: an AsyncCheckpointer with the "
                    "/dev/shm tier whose snapshot buffer is prepared in the background from before step 1 (the "
                    "trainer's first launch)")
    ap.add_argument("--save-after", type=int, default=-1, help="save after this step (0-based)")
    ap.add_argument("--save-dir", default=None, help="checkpoint dir (shared by a --kill-after-save run and a "
                    "--resume run: the /dev/shm snapshot outlives the killed process, as in the SIGKILL drill)")
    ap.add_argument("--kill-after-save", action="store_true", help="SIGKILL this process right after the save")
    ap.add_argument("--resume", action="store_true", help="restore from --save-dir before step 1 (the snapshot "
                    "buffer is then prepared after the first step, as the trainer does after a restore)")
    ap.add_argument("--headroom", type=float, default=None, help="EngineConfig.hbm_headroom")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    t_imp0 = time.time()
    import torch
    from distributed_llm_training_gpu_manager_amd.models import get_config
    from distributed_llm_training_gpu_manager_amd.parallel.comm import ShadowComm
    from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine
    from distributed_llm_training_gpu_manager_amd import _native
    _native.hip_ops()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    rec = {"model": a.model, "seq": a.seq, "shadow_world": a.shadow_world, "ckpt": bool(a.ckpt), "warm": a.warm,
           "import_s": round(time.time() - t_imp0, 2)}
    mc = get_config(a.model, **({"n_layers": a.n_layers} if a.n_layers else {}))
    ec = EngineConfig(zero_stage=3, micro_batch_size=1, seq_len=a.seq, grad_accum=1, lr=3e-5,
                      activation_checkpointing=bool(a.ckpt),
                      **({"hbm_headroom": a.headroom} if a.headroom is not None else {}))
    t0 = time.time()
    eng = ZeroEngine(mc, ec, dev, ShadowComm(a.shadow_world, 0, async_mode=True))
    torch.cuda.synchronize()
    rec["engine_s"] = round(time.time() - t0, 2)
    if a.warm != "none":
        t0 = time.time()
        info = eng.warm_up()
        torch.cuda.synchronize()
        rec["warm_s"] = round(time.time() - t0, 2)
        rec["warm_info"] = info
    ck = None
    if a.ckpt_tier == "shm":
        import tempfile
        from distributed_llm_training_gpu_manager_amd.ckpt.checkpoint import AsyncCheckpointer
        ck = AsyncCheckpointer(eng, a.save_dir or tempfile.mkdtemp(prefix="probe_ck_"), shm=True, disk=False,
                               keep_last=1)
        rec["ckpt_mode"] = ck.mode
        if a.resume:
            t0 = time.time()
            cs = ck.load("auto")
            torch.cuda.synchronize()
            rec["restore_s"] = round(time.time() - t0, 2)
            rec["restored_from"] = ck.restored_from
            rec["restore_stats"] = getattr(ck, "restore_stats", {})
            rec["resumed"] = cs is not None
        else:
            t0 = time.time()
            ck.prepare_async()
            rec["prepare_started_s"] = round(time.time() - t0, 3)
    unit_t = {}
    cur = {"step": 0}
    if a.per_unit:
        for si, (unit, _) in enumerate(eng.stages):
            f0, b0 = unit.forward, unit.backward

            def fwd(p, x, ctx, _f=f0, _si=si):
                torch.cuda.synchronize()
                t = time.time()
                out = _f(p, x, ctx)
                torch.cuda.synchronize()
                unit_t.setdefault((cur["step"], "f"), []).append((time.time() - t, _si))
                return out

            def bwd(p, g, saved, dy, ctx, _b=b0, _si=si):
                torch.cuda.synchronize()
                t = time.time()
                out = _b(p, g, saved, dy, ctx)
                torch.cuda.synchronize()
                unit_t.setdefault((cur["step"], "b"), []).append((time.time() - t, _si))
                return out
            unit.forward, unit.backward = fwd, bwd
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    steps = []
    for s in range(a.steps):
        cur["step"] = s
        toks = torch.randint(0, mc.vocab_size, (1, a.seq + 1), device=dev, generator=gen)
        torch.cuda.synchronize()
        t0 = time.time()
        eng.train_step([(toks[:, :-1].contiguous(), toks[:, 1:].contiguous())])
        torch.cuda.synchronize()
        st = torch.cuda.memory_stats(dev)
        steps.append({"step_s": round(time.time() - t0, 3),
                      "reserved_GiB": round(torch.cuda.memory_reserved(dev) / 2 ** 30, 1),
                      "segments": int(st.get("segment.all.current", 0)),
                      "alloc_retries": int(st.get("num_alloc_retries", 0)),
                      "peak_alloc_GiB": round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 1),
                      "hip_mallocs": int(st.get("segment.all.allocated", 0)),
                      "prep_alive": bool(ck is not None and ck._prep is not None and ck._prep.is_alive())})
        if ck is not None and a.resume and s == 0:
            ck.prepare_async()  # after the first recovered step, as the trainer does
        if ck is not None and s == a.save_after:
            t0 = time.time()
            ck.save(s + 1, blocking=True)
            steps[-1]["save_s"] = round(time.time() - t0, 2)
            steps[-1]["save_rec"] = {k: v for k, v in (ck.history[-1] if ck.history else {}).items()}
            steps[-1]["prep_stats"] = dict(ck.prep_stats)
            if a.kill_after_save:
                rec["steps"] = steps
                print(json.dumps(rec), flush=True)
                if a.out:
                    with open(a.out, "w") as f:
                        json.dump(rec, f, indent=1)
                import signal
                os.kill(os.getpid(), signal.SIGKILL)
    rec["steps"] = steps
    if ck is not None:
        t0 = time.time()
        ck.close(discard_shm=True)
        rec["close_s"] = round(time.time() - t0, 2)
    if unit_t:
        rec["units"] = {f"step{st}_{ph}": {"total_s": round(sum(t for t, _ in v), 3), "calls": len(v),
                                           "worst": [(round(t, 3), si) for t, si in sorted(v, reverse=True)[:4]]}
                        for (st, ph), v in sorted(unit_t.items())}
        rec["n_units"] = len(eng.stages)
    print(json.dumps(rec), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rec, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
