"""Correctness checks a multi-GPU run makes on itself before it measures a transport.

The xGMI mesh (parallel/xgmi_mesh.py) and RCCL are exercised across real devices for the first time by the
round driver's 8-GPU scaling run, so that run checks -- on the same inputs, on every rank -- that

* ``all_gather``: the mesh pull == RCCL ``all_gather_into_tensor``, bit for bit;
* ``reduce_scatter``: the mesh push + fp32 rank-order reduce == the same sum computed locally from every rank's
  input fetched over RCCL (bit for bit), and within bf16 rounding of RCCL's own reduce-scatter;
* ``ep_dispatch_combine``: the dropless mesh EP exchange == the RCCL dispatcher (``ExpertDispatcher``) for every
  row of a skewed routing (dispatch, combine, redispatch), no overflow;
* ``zero3_parity``: two steps of llama-tiny ZeRO-3 on RCCL and on the mesh, each against one process training the
  same global batch (the engine's multi-rank tolerance) and against each other.

Every rank runs every check (they are collective); the verdict is the AND over ranks. ``tools/mesh_sweep.py``
(bench.py's post-result child) prints it as one ``[mesh-check] {...}`` line on stderr. Without a GPU only the
parity of the gloo ranks against one process runs (the mesh needs device memory): the same code the GPU tests
drive with ranks sharing one MI355X.
"""
from __future__ import annotations

from typing import Any, Dict, List

import torch
import torch.distributed as dist

from ..parallel.comm import Comm, ShadowComm


def _vec(seed: int, n: int, dtype=torch.float32, device="cpu") -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, generator=g).to(dtype).to(device)


def _all_ranks_ok(ok: bool, device) -> bool:
    if not dist.is_initialized():
        return ok
    dev = device if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([1.0 if ok else 0.0], device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item() > 0.5)


def check_all_gather(comm: Comm, device, n: int = 1 << 20) -> Dict[str, Any]:
    from ..parallel.xgmi_mesh import XgmiMesh
    W, r = comm.world, comm.rank
    mesh = XgmiMesh(comm, device, {"p16": (n * 2, 1)}, timeout_s=60.0)
    try:
        shard = mesh.region_tensor("p16", torch.bfloat16, n)
        mesh.quiesce()
        shard.copy_(_vec(7000 + r, n, torch.bfloat16, device))
        mesh.publish()
        got = torch.empty(W * n, dtype=torch.bfloat16, device=device)
        mesh.all_gather_pull(got, shard)
        ref = torch.empty_like(got)
        comm.all_gather(ref, shard.clone(), async_op=False).wait()
        torch.cuda.synchronize(device)
        mesh.check()
        ok = torch.equal(got, ref)
        return {"pass": _all_ranks_ok(ok, device), "alloc_mode": mesh.alloc_mode, "elems": W * n}
    finally:
        mesh.close()


def check_reduce_scatter(comm: Comm, device, n: int = 1 << 20) -> Dict[str, Any]:
    """The two reduce-scatters the engine issues, mesh against RCCL on the same inputs:

    * bf16 (per-micro-batch scratch path): the mesh's rank-order fp32 sum of the bf16-rounded chunks must equal that
      expression bit for bit; RCCL's bf16 ring rounds at every hop, so it agrees within bf16 rounding (2e-2);
    * fp32 (the once-per-step reduce of the local accumulator, the default): both transports sum the same fp32 values,
      only the order of the additions differs -- within fp32 rounding (1e-5 relative)."""
    from ..parallel.xgmi_mesh import XgmiMesh, rs_region_bytes
    W, r = comm.world, comm.rank
    mesh = XgmiMesh(comm, device, {"rs": (rs_region_bytes(W, n, 4), 2)}, timeout_s=60.0)
    try:
        x = _vec(9000 + r, W * n, torch.float32, device)
        out = torch.zeros(n, dtype=torch.float32, device=device)
        scale = 1.0 / W
        mesh.reduce_scatter(out, x, scale, False)
        # reference: every rank's bf16-rounded chunk `r`, summed in fp32 in rank order, times the scale
        xb = x.to(torch.bfloat16)
        allx = torch.empty(W * W * n, dtype=torch.bfloat16, device=device)
        comm.all_gather(allx, xb, async_op=False).wait()
        chunks = allx.view(W, W, n)[:, r].float()
        ref = chunks[0].clone()
        for s in range(1, W):
            ref = ref + chunks[s]
        ref = ref * torch.tensor(scale, dtype=torch.float32, device=device)
        # RCCL's own bf16 reduce-scatter (its order and precision): within bf16 rounding of the exact sum
        rccl = torch.empty(n, dtype=torch.bfloat16, device=device)
        comm.reduce_scatter(rccl, xb, avg=True, async_op=False).wait()
        # fp32 slots against RCCL's fp32 reduce-scatter
        out32 = torch.zeros(n, dtype=torch.float32, device=device)
        mesh.reduce_scatter(out32, x, scale, False, fp32=True)
        rccl32 = torch.empty(n, dtype=torch.float32, device=device)
        comm.reduce_scatter(rccl32, x, avg=True, async_op=False).wait()
        torch.cuda.synchronize(device)
        mesh.check()
        exact = torch.equal(out, ref)
        rel = float((rccl.float() - out).abs().max() / out.abs().max().clamp_min(1e-8))
        rel32 = float((rccl32 - out32).abs().max() / out32.abs().max().clamp_min(1e-8))
        ok = exact and rel < 2e-2 and rel32 < 1e-5
        return {"pass": _all_ranks_ok(ok, device), "bit_exact_vs_rank_order_fp32": exact,
                "max_rel_vs_rccl_bf16": round(rel, 5), "max_rel_fp32_mesh_vs_rccl_fp32": rel32}
    finally:
        mesh.close()


def check_ep_exchange(comm: Comm, device, T: int = 512, K: int = 2, D: int = 1024, E: int = 0) -> Dict[str, Any]:
    from ..ops.moe import moe_permute
    from ..parallel.ep import ExpertDispatcher, MeshExpertDispatcher
    W, r = comm.world, comm.rank
    E = E or 2 * W
    ref = ExpertDispatcher(comm, E)
    mesh = MeshExpertDispatcher(comm, E, device, T * K, D, torch.bfloat16, capacity_factor=None, timeout_s=60.0)
    ok, worst, msgs = True, 0, []
    try:
        for it, skew in enumerate((False, True)):
            g = torch.Generator().manual_seed(31 * it + 101 * r)
            if skew:  # nearly every slot to expert 0: its owner receives far more than the balanced share
                topi = torch.zeros(T, K, dtype=torch.long)
                topi[:, 1] = 1 + torch.randint(0, E - 1, (T,), generator=g)
            else:
                topi = torch.rand(T, E, generator=g).topk(K, dim=-1).indices
            topi = topi.to(device)
            offsets, pos, tok = moe_permute(topi, E)
            counts = (offsets[1:] - offsets[:-1]).long()
            x = _vec(3000 + 7 * it + r, T * K * D, torch.bfloat16, device).view(T * K, D)
            xr, cr = ref.dispatch(x, counts, offsets)
            xm, cm = mesh.dispatch(x, counts, offsets)
            n = xr.shape[0]
            worst = max(worst, n)
            if int(cm.nrows) != n or not torch.equal(xm[:n], xr):
                ok = False
                msgs.append(f"dispatch {'skew' if skew else 'uniform'}")
            yr = xr * 3 + 1
            ym = torch.zeros_like(xm)
            ym[:n] = xm[:n] * 3 + 1
            if not torch.equal(mesh.combine(ym, cm), ref.combine(yr, cr)):
                ok = False
                msgs.append(f"combine {'skew' if skew else 'uniform'}")
            dy = _vec(5000 + 7 * it + r, T * K * D, torch.bfloat16, device).view(T * K, D)
            if not torch.equal(mesh.redispatch(dy, cm)[:n], ref.redispatch(dy, cr)):
                ok = False
                msgs.append(f"redispatch {'skew' if skew else 'uniform'}")
        torch.cuda.synchronize(device)
        mesh.mesh.check()
        if mesh.overflowed():
            ok = False
            msgs.append("overflow word set (dropless)")
        return {"pass": _all_ranks_ok(ok, device), "max_rows_received": worst, "capacity_rows": mesh.C,
                "errors": msgs}
    finally:
        mesh.close()


def _parity_run(comm, device, W: int, rank: int, mesh: bool, steps: int, ga: int, world1: bool):
    from ..models import get_config
    from ..parallel.zero import EngineConfig, ZeroEngine
    mc = get_config("llama-tiny")
    cfg = EngineConfig(zero_stage=3, micro_batch_size=2, seq_len=128, grad_accum=ga * (W if world1 else 1),
                       lr=5e-3, scheduler="constant", init_device="cpu", grad_clip=1.0,
                       xgmi_mesh="on" if mesh else "off", mesh_timeout_s=60.0)
    eng = ZeroEngine(mc, cfg, device, ShadowComm(1, 0) if world1 else comm)
    g = torch.Generator().manual_seed(23)
    data = [[torch.randint(0, mc.vocab_size, (2, 129), generator=g) for _ in range(W * ga)] for _ in range(steps)]
    grads0 = None
    for step in data:
        mine = step if world1 else step[rank * ga:(rank + 1) * ga]
        eng.train_step([(t[:, :-1].contiguous().to(device), t[:, 1:].contiguous().to(device)) for t in mine])
        if grads0 is None:
            grads0 = {k: v.float().cpu() for k, v in eng.full_grads().items()}
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    if eng.mesh is not None:
        eng.check_transport()
    params = {k: v.float().cpu() for k, v in eng.full_params().items()}
    issued = eng.mesh.issued if eng.mesh is not None else 0
    for m in (eng.mesh, eng.ep_mesh):
        if m is not None:
            m.close()
    return grads0, params, issued


def _parity(a, b) -> Dict[str, float]:
    (ga_, pa, _), (gb, pb, _) = a, b
    gerr = max(float((ga_[k] - gb[k]).abs().max() / gb[k].abs().max().clamp_min(1e-8)) for k in gb)
    pmax = max(float((pa[k] - pb[k]).abs().max()) for k in pb)
    return {"grad_max_rel": round(gerr, 5), "param_max_abs": round(pmax, 6)}


def check_zero3_parity(comm: Comm, device, mesh: bool, steps: int = 2, ga: int = 2) -> Dict[str, Any]:
    """llama-tiny ZeRO-3, `steps` optimizer steps: RCCL (and the mesh, on the GPU) against one process on the same
    global batch. Tolerance = the engine's multi-rank tests (bf16 gradient reductions vs one process)."""
    W, r = comm.world, comm.rank
    runs = {"rccl": _parity_run(comm, device, W, r, False, steps, ga, False)}
    if mesh:
        runs["mesh"] = _parity_run(comm, device, W, r, True, steps, ga, False)
    ref = _parity_run(comm, device, W, r, False, steps, ga, True)  # every rank: the world-1 reference
    out: Dict[str, Any] = {}
    ok = True
    for name, run in runs.items():
        d = _parity(run, ref)
        good = d["grad_max_rel"] < 3e-2 and d["param_max_abs"] <= 2 * 5e-3 * steps + 1e-3
        out[f"{name}_vs_world1"] = {**d, "pass": good}
        ok &= good
    if mesh:
        d = _parity(runs["mesh"], runs["rccl"])
        # both reduce the same fp32 local gradients (step_comm_dtype fp32): only the order of the fp32 additions
        # differs, so the reduced gradients agree to fp32 rounding, not merely to bf16 rounding
        d["pass"] = d["grad_max_rel"] < 1e-4
        out["mesh_vs_rccl"] = d
        out["mesh_collectives_issued"] = runs["mesh"][2]
        ok &= runs["mesh"][2] > 0 and d["pass"]
    out["pass"] = _all_ranks_ok(ok, device)
    return out


def run_checks(comm: Comm, device) -> Dict[str, Any]:
    """Every check that applies to this device; each failure is recorded, never raised."""
    rec: Dict[str, Any] = {"world": comm.world, "backend": comm.backend, "device": str(device)}
    gpu = device.type == "cuda"
    checks: List = []
    if gpu and comm.world > 1:
        checks += [("all_gather", lambda: check_all_gather(comm, device)),
                   ("reduce_scatter", lambda: check_reduce_scatter(comm, device)),
                   ("ep_dispatch_combine", lambda: check_ep_exchange(comm, device))]
    else:
        rec["mesh_ops"] = "skipped (the mesh needs GPU memory)"
    checks.append(("zero3_parity", lambda: check_zero3_parity(comm, device, mesh=gpu and comm.world > 1)))
    for name, fn in checks:
        try:
            rec[name] = fn()
        except Exception as e:  # noqa: BLE001 -- reported, the caller decides
            rec[name] = {"pass": False, "error": f"{type(e).__name__}: {e}"[:300]}
    rec["alloc_mode"] = rec.get("all_gather", {}).get("alloc_mode")
    rec["pass"] = all(v.get("pass", False) for k, v in rec.items() if isinstance(v, dict))
    return rec
