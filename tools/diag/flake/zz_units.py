"""Round-5 flake probe, second stage: the per-op synchronising digest hides the mismatch (a race), so this one
snapshots every unit's outputs and gradients with device-side clones on the issuing stream (no host sync) and,
after three engines, names the first (micro-batch, stage, phase, tensor) where engine 0 differs from engine 1.
Appended to tests/test_shadow_async_gpu.py on the box by tools/diag/r05/units.sh."""


def _zz_snap_units(eng, log):
    import torch

    def clone(x):
        if isinstance(x, torch.Tensor):
            return x.detach().clone()
        if isinstance(x, (tuple, list)):
            return type(x)(clone(v) for v in x)
        return None

    for si, (unit, gis) in enumerate(eng.stages):
        if getattr(unit, "_zz_wrapped", False):
            continue
        unit._zz_wrapped = True
        f0, b0 = unit.forward, unit.backward

        def fwd(p, x, ctx, _f=f0, _si=si):
            y, saved = _f(p, x, ctx)
            log.append(("fwd", ctx.micro_index, _si, clone(y)))
            return y, saved

        def bwd(p, g, saved, dy, ctx, _b=b0, _si=si):
            dx = _b(p, g, saved, dy, ctx)
            log.append(("bwd", ctx.micro_index, _si, clone(dx)))
            log.append(("grad", ctx.micro_index, _si, {k: v.detach().clone() for k, v in g.items()}))
            return dx
        unit.forward, unit.backward = fwd, bwd


def _zz_patch_moe(log):
    """MixtralBlock.moe_forward with a device-side clone of every intermediate (same ops, same order)."""
    import torch
    from distributed_llm_training_gpu_manager_amd import ops
    from distributed_llm_training_gpu_manager_amd.models import mixtral as mx

    import os
    taps = set(os.environ.get("ZZ_TAP", "").split(","))
    _log = log

    class _L:
        @staticmethod
        def append(rec):
            if rec[0].split(".", 1)[1] in taps:
                _log.append(rec)
    log = _L

    def moe_forward(self, p, hn2, ctx):
        c = self.cfg
        T, E, K = hn2.shape[0], c.n_experts, c.top_k
        logits = torch.mm(hn2, p["router"].t())
        log.append(("moe.logits", ctx.micro_index, self.layer, logits.detach().clone()))
        probs, topi, gates = ops.router_topk(logits, K)
        log.append(("moe.router", ctx.micro_index, self.layer, [probs.clone(), topi.clone(), gates.clone()]))
        offsets, pos, tok = mx.moe_permute(topi, E)
        log.append(("moe.permute", ctx.micro_index, self.layer, [offsets.clone(), pos.clone(), tok.clone()]))
        counts = (offsets[1:] - offsets[:-1]).long()
        x_sorted = hn2.index_select(0, tok)
        disp = self.dispatcher(ctx)
        x_local, dctx = disp.dispatch(x_sorted, counts, offsets)
        log.append(("moe.x_local", ctx.micro_index, self.layer, [x_local.clone(), dctx.local_offsets.clone()]))
        y_local, exp_saved = self._experts_fwd(p, x_local, dctx)
        log.append(("moe.experts", ctx.micro_index, self.layer, [exp_saved[0].clone(), exp_saved[1].clone(),
                                                                 y_local.clone()]))
        y_sorted = disp.combine(y_local, dctx)
        log.append(("moe.y_sorted", ctx.micro_index, self.layer, y_sorted.clone()))
        out = mx.moe_combine(y_sorted, pos, gates)
        log.append(("moe.out", ctx.micro_index, self.layer, out.clone()))
        f = counts.float() / float(T * K) * K
        ctx.aux.setdefault("moe_aux", []).append(float(E) * (f * probs.mean(0)).sum())
        return out, (probs, topi, gates, pos, f, x_local, dctx, exp_saved, y_sorted)
    mx.MixtralBlock.moe_forward = moe_forward


def _zz_cmp(a, b):
    import torch
    if a is None or b is None:
        return None
    if isinstance(a, torch.Tensor):
        if a.shape != b.shape:
            return "shape"
        d = (a.float() - b.float()).abs()
        n = int((d > 0).sum()) + int((a.float().isnan() != b.float().isnan()).sum())
        return None if n == 0 else {"n": n, "max": float(torch.nan_to_num(d, nan=-1).max()), "numel": a.numel()}
    if isinstance(a, dict):
        out = {k: _zz_cmp(a[k], b[k]) for k in a}
        out = {k: v for k, v in out.items() if v is not None}
        return out or None
    out = [_zz_cmp(x, y) for x, y in zip(a, b)]
    return out if any(o is not None for o in out) else None


def test_zz_units():
    import json
    import os
    import torch
    from distributed_llm_training_gpu_manager_amd.models import get_config
    from distributed_llm_training_gpu_manager_amd.parallel.comm import ShadowComm
    from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine
    dev = torch.device("cuda", 0)
    var = os.environ.get("ZZ_VAR", "")
    if var == "rocblas":
        torch.backends.cuda.preferred_blas_library("cublas")  # torch.mm through rocBLAS instead of hipBLASLt
    if var == "prio":  # the shadow comm streams from the high-priority pool: never the side streams' HIP streams
        _orig_run = ShadowComm._run

        def _run(self, fn, tensors, async_op):
            if self._stream is None and tensors and tensors[0].is_cuda:
                self._stream = torch.cuda.Stream(tensors[0].device, priority=-1)
            return _orig_run(self, fn, tensors, async_op)
        ShadowComm._run = _run
    streams = []
    logs = []
    holder = []
    _zz_patch_moe(holder)
    states = []
    for run in range(3):
        mc = get_config("mixtral-tiny")
        ec = EngineConfig(micro_batch_size=2, seq_len=64, grad_accum=2, lr=1e-3, scheduler="constant", grad_clip=1.0,
                          zero_stage=3, expert_parallel_size=4, local_grad_accum=False, optimizer_overlap=False)
        eng = ZeroEngine(mc, ec, dev, ShadowComm(4, 0, async_mode=True, delay_cycles=200_000))
        log = holder
        log.clear()
        _zz_snap_units(eng, log)
        g = torch.Generator().manual_seed(3)
        for step in range(3):
            mbs = []
            for _ in range(2):
                t = torch.randint(0, mc.vocab_size, (2, 65), generator=g).to(dev)
                mbs.append((t[:, :-1].contiguous(), t[:, 1:].contiguous()))
            eng.train_step(mbs)
            log.append(("opt", step, -1, {"master": eng.master.detach().clone(), "grad": eng.grad_shard.detach().clone()}))
        torch.cuda.synchronize()
        from distributed_llm_training_gpu_manager_amd.utils.streams import _STREAMS
        cs = {}
        for nm in ("comm", "gather_comm", "ep_comm", "edp_comm"):
            c = getattr(eng, nm, None)
            st = getattr(c, "_stream", None) if c is not None else None
            cs[nm] = st.cuda_stream if st is not None else None
        cs.update({f"side:{k[1]}": v.cuda_stream for k, v in _STREAMS.items()})
        streams.append(cs)
        logs.append(list(log))
        states.append(eng.master.detach().cpu().clone())
        del eng
    rep = {"state_equal": {"01": torch.equal(states[0], states[1]), "12": torch.equal(states[1], states[2])},
           "entries": len(logs[0]), "first": [], "streams": streams, "var": var}
    for i, (a, b) in enumerate(zip(logs[0], logs[1])):
        c = _zz_cmp(a[3], b[3])
        if c is not None:
            rep["first"].append({"i": i, "phase": a[0], "micro": a[1], "stage": a[2], "diff": c})
            if len(rep["first"]) >= 10:
                break
    out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "digest")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "units_report.json"), "w") as f:
        json.dump(rep, f, indent=1, default=str)
    print(json.dumps(rep, default=str)[:3000])
