"""The device-driven xGMI mesh transport (parallel/xgmi_mesh.py, csrc/kernels/xgmi_mesh.hip) and the EP dispatcher
built on it (parallel/ep.py MeshExpertDispatcher).

Ranks share one MI355X here (IPC within one device; gloo carries the handle exchange -- RCCL refuses two ranks on
one GPU). Every rank maps every peer's heap and the kernels move data and flags exactly as on an 8-GPU node; only
the wire differs. Checks, all bit-exact:
* all-gather (pull): == concatenation of every rank's shard, over several versions (quiesce / publish ordering);
* reduce-scatter (push + fp32 reduce): == the fp32 rank-order sum of the bf16-rounded chunks, times the scale,
  (+ the previous value when accumulating), from fp32 and from bf16 inputs, several epochs through 2 slots;
* EP dispatch / redispatch / combine: == the RCCL-path dispatcher (ExpertDispatcher over the same ranks) for EVERY
  row, with an expert that receives no rows and with a skewed routing that sends nearly every row to one owner
  (dropless: the receive slot holds the worst case), both with a static worst-case output and with the output sized
  by one host read; an explicit capacity that is too small raises the overflow word (an assertion: the engine stops
  the job) and its rows past the capacity come back as zeros;
* the MoE EP micro-batch path replays from a captured HIP graph.
"""
import os
import socket
import warnings

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    return dev


def _finish(rank, ok, out_path, extra=None):
    flag = torch.tensor([1 if ok else 0])
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if rank == 0:
        torch.save({"ok": int(flag), **(extra or {})}, out_path)
    dist.barrier()
    dist.destroy_process_group()


def _vec(seed, n, dtype=torch.bfloat16):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, generator=g).to(dtype)


def _zero_worker(rank, world, port, n, iters, out_path):
    dev = _init(rank, world, port)
    from distributed_llm_training_gpu_manager_amd.parallel.comm import Comm
    from distributed_llm_training_gpu_manager_amd.parallel.xgmi_mesh import XgmiMesh, rs_region_bytes
    mesh = XgmiMesh(Comm(), dev, {"p16": (n * 2, 1), "rs": (rs_region_bytes(world, n), 2)}, timeout_s=20)
    shard = mesh.region_tensor("p16", torch.bfloat16, n)
    ok = True
    msgs = []
    for it in range(iters):
        # optimizer-style update of this rank's partition: quiesce (peers done with the old version), write, publish
        mesh.quiesce()
        shard.copy_(_vec(1000 * it + rank, n).to(dev))
        mesh.publish()
        out = torch.empty(world * n, dtype=torch.bfloat16, device=dev)
        mesh.all_gather_pull(out, shard)
        want = torch.cat([_vec(1000 * it + r, n) for r in range(world)])
        if not torch.equal(out.cpu(), want):
            ok = False
            msgs.append(f"ag it{it}")
        # reduce-scatter from fp32 (cast on the fly) and from bf16, accumulating into an fp32 shard
        for src_dtype in (torch.float32, torch.bfloat16):
            xs = [_vec(7 * it + 100 * r + 1, world * n, torch.float32) for r in range(world)]
            if src_dtype == torch.bfloat16:
                xs = [x.to(torch.bfloat16) for x in xs]
            prev = _vec(99 + rank + it, n, torch.float32)
            acc = it % 2 == 1
            scale = 1.0 / world
            o = prev.clone().to(dev)
            mesh.reduce_scatter(o, xs[rank].to(dev), scale, acc)
            chunks = [x.to(torch.bfloat16).float()[rank * n:(rank + 1) * n] for x in xs]
            ref = chunks[0].clone()
            for c in chunks[1:]:
                ref = ref + c
            ref = ref * torch.tensor(scale, dtype=torch.float32)
            if acc:
                ref = prev + ref
            if not torch.equal(o.cpu(), ref):
                ok = False
                msgs.append(f"rs it{it} {src_dtype} maxdiff {float((o.cpu() - ref).abs().max())}")
    torch.cuda.synchronize()
    mesh.check()
    mode = mesh.alloc_mode
    mesh.close()
    _finish(rank, ok, out_path, {"msgs": msgs, "mode": mode} if rank == 0 else None)


@pytest.mark.parametrize("world,n", [(2, 4096), (4, 1 << 18)])
def test_mesh_all_gather_and_reduce_scatter_bit_exact(tmp_path, world, n):
    out = str(tmp_path / "mesh.pt")
    mp.spawn(_zero_worker, args=(world, _free_port(), n, 4, out), nprocs=world, join=True)
    res = torch.load(out, weights_only=True)
    assert res["ok"] == 1, res.get("msgs")
    # which memory kind the driver exported (uncached is the design point; the fallbacks are recorded)
    warnings.warn(f"xGMI mesh heap allocated {res['mode']}")


def _routing(rank, T, K, E, seed, skew):
    g = torch.Generator().manual_seed(seed + 17 * rank)
    if skew:  # nearly every slot to expert 0: the owner of expert 0 overflows its capacity
        topi = torch.zeros(T, K, dtype=torch.long)
        topi[:, 1] = 1 + torch.randint(0, E - 2, (T,), generator=g)
    else:  # expert E-1 never chosen (an empty expert on its owner)
        scores = torch.rand(T, E - 1, generator=g)
        topi = scores.topk(K, dim=-1).indices
    return topi


def _ep_worker(rank, world, port, E, T, K, D, factor, skew, sized, out_path):
    dev = _init(rank, world, port)
    from distributed_llm_training_gpu_manager_amd.ops.moe import moe_permute
    from distributed_llm_training_gpu_manager_amd.parallel.comm import Comm
    from distributed_llm_training_gpu_manager_amd.parallel.ep import ExpertDispatcher, MeshExpertDispatcher
    comm = Comm()
    ref = ExpertDispatcher(comm, E)
    mesh = MeshExpertDispatcher(comm, E, dev, T * K, D, torch.bfloat16, capacity_factor=factor, timeout_s=20,
                                sized_output=sized)
    C = mesh.C
    if factor is None and C < world * T * K:
        ok_geom = False
    else:
        ok_geom = True
    ok, msgs = True, []
    for it in range(3):
        topi = _routing(rank, T, K, E, 100 * it, skew).to(dev)
        offsets, pos, tok = moe_permute(topi, E)
        counts = (offsets[1:] - offsets[:-1]).long()
        x = _vec(1000 * it + rank, T * K * D).view(T * K, D).to(dev)
        xr, cr = ref.dispatch(x, counts, offsets)
        xm, cm = mesh.dispatch(x, counts, offsets)
        total = xr.shape[0]
        keep = min(total, C)
        if factor is None and (keep != total or xm.shape[0] < total):  # dropless: every row arrives
            ok = False
            msgs.append(f"dropless dispatch lost rows: total {total} C {C} out rows {xm.shape[0]}")
        if sized and xm.shape[0] != max(64, (total + 63) // 64 * 64):
            ok = False
            msgs.append(f"sized output {xm.shape[0]} rows for {total}")
        if int(cm.nrows) != keep or not torch.equal(xm[:keep].cpu(), xr[:keep].cpu()):
            ok = False
            msgs.append(f"dispatch it{it} total {total} C {C} nrows {int(cm.nrows)}")
        want_off = torch.clamp(cr.local_offsets.cpu(), max=C)
        if not torch.equal(cm.local_offsets.cpu(), want_off):
            ok = False
            msgs.append(f"offsets it{it} {cm.local_offsets.tolist()} vs {want_off.tolist()}")
        # an "expert" computation on the valid rows; rows past the capacity were never received -> zero back
        yr = xr * 3 + 1
        yr[keep:] = 0
        ym = torch.zeros_like(xm)
        ym[:keep] = xm[:keep] * 3 + 1
        outr = ref.combine(yr, cr)
        outm = mesh.combine(ym, cm)
        if not torch.equal(outm.cpu(), outr.cpu()):
            ok = False
            msgs.append(f"combine it{it}")
        dy = _vec(5000 + 1000 * it + rank, T * K * D).view(T * K, D).to(dev)
        dr = ref.redispatch(dy, cr)
        dm = mesh.redispatch(dy, cm)
        if not torch.equal(dm[:keep].cpu(), dr[:keep].cpu()):
            ok = False
            msgs.append(f"redispatch it{it}")
    torch.cuda.synchronize()
    mesh.mesh.check()
    ovf = mesh.overflowed()
    want_ovf = bool(skew) and factor is not None
    if ovf != want_ovf or not ok_geom:
        ok = False
        msgs.append(f"overflow flag {ovf} (skew {skew}, factor {factor}, C {C})")
    mesh.close()
    _finish(rank, ok, out_path, {"msgs": msgs} if rank == 0 else None)


@pytest.mark.parametrize("world,E,factor,skew,sized", [
    (2, 4, None, False, False), (4, 8, None, False, False), (4, 4, None, False, True),
    (4, 8, None, True, False), (4, 8, None, True, True),  # skewed routing, dropless: every row, bit-exact
    (4, 8, 0.5, True, False)])  # explicit capacity: the overflow word is raised (the engine raises on it)
def test_mesh_expert_dispatch_matches_rccl_dispatcher(tmp_path, world, E, factor, skew, sized):
    out = str(tmp_path / "ep.pt")
    mp.spawn(_ep_worker, args=(world, _free_port(), E, 96, 2, 128, factor, skew, sized, out), nprocs=world,
             join=True)
    res = torch.load(out, weights_only=True)
    assert res["ok"] == 1, res.get("msgs")


def _check_worker(rank, world, port, out_path):
    dev = _init(rank, world, port)
    import json
    from distributed_llm_training_gpu_manager_amd.parallel.comm import Comm
    from distributed_llm_training_gpu_manager_amd.utils.meshcheck import run_checks
    rec = run_checks(Comm(), dev)
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(rec, f)
    dist.barrier()
    dist.destroy_process_group()


def test_mesh_self_check_passes_with_ranks_sharing_one_gpu(tmp_path):
    """The checks the multi-GPU bench runs on itself before its mesh sweep (utils/meshcheck.py):
    the same code, two ranks on one MI355X (gloo for the bootstrap and as the "RCCL" side)."""
    import json
    out = str(tmp_path / "check.json")
    mp.spawn(_check_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    with open(out) as f:
        rec = json.load(f)
    assert rec["pass"], json.dumps(rec)[:6000]
    assert rec["all_gather"]["pass"] and rec["reduce_scatter"]["bit_exact_vs_rank_order_fp32"], rec
    ep = rec["ep_dispatch_combine"]
    assert ep["pass"] and ep["max_rows_received"] > 512 * 2, ep  # the skewed routing exceeded the balanced share
    par = rec["zero3_parity"]
    assert par["rccl_vs_world1"]["pass"] and par["mesh_vs_world1"]["pass"] and par["mesh_collectives_issued"] > 0


@pytest.mark.gpu
def test_shadow_mesh_heaps_are_pooled_not_freed():
    """A dead mesh's heap goes back to a process-lifetime pool and the next mesh of that memory kind reuses one, zeroed:
    an uncached heap is never returned to the driver (freeing one made later engines in the process compute different
    bits; README "Determinism")."""
    import gc
    from distributed_llm_training_gpu_manager_amd.parallel import xgmi_mesh as X
    from distributed_llm_training_gpu_manager_amd.parallel.comm import ShadowComm

    dev = torch.device("cuda", 0)
    m = X.XgmiMesh(ShadowComm(4, 0), dev, {"rs": (1 << 20, 2)})
    ptr, key = m.heap.data_ptr(), (0, X.ALLOC_MODES.index(m.alloc_mode))
    m.heap[:m.heap_bytes].fill_(7)
    del m
    gc.collect()
    pooled = {h.data_ptr() for h in X._HEAP_POOL.get(key, [])}
    assert ptr in pooled  # returned, not freed
    m2 = X.XgmiMesh(ShadowComm(4, 0), dev, {"rs": (1 << 19, 2)})  # smaller: a pooled heap fits
    assert m2.heap.data_ptr() in pooled
    assert int(m2.heap[:m2.heap_bytes].count_nonzero()) == 0
    del m2
    gc.collect()
