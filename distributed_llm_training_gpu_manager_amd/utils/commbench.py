"""RCCL collective bus-bandwidth measurement (rccl-tests conventions), shared by tools/comm_bench.py and
the multi-GPU bench (bench.py measures the xGMI curve after its timed steps when WORLD_SIZE > 1).

algbw = bytes / time; busbw = algbw * (W-1)/W for all_gather / reduce_scatter / all_to_all and
2(W-1)/W for all_reduce. The slowest rank defines each collective's time.
"""
from __future__ import annotations

import time
from typing import Dict, List, Sequence

import torch

from ..parallel.comm import DONE, Comm

FACTOR = {"all_gather": lambda w: (w - 1) / w, "ipc_mesh_all_gather": lambda w: (w - 1) / w,
          "reduce_scatter": lambda w: (w - 1) / w, "ipc_mesh_reduce_scatter": lambda w: (w - 1) / w,
          "all_to_all": lambda w: (w - 1) / w, "ipc_mesh_all_to_all": lambda w: (w - 1) / w,
          "all_reduce": lambda w: 2 * (w - 1) / w}
MESH_OPS = ("ipc_mesh_all_gather", "ipc_mesh_reduce_scatter", "ipc_mesh_all_to_all")


def run(op: str, comm: Comm, nbytes: int, device, dtype, iters: int, warmup: int) -> float:
    mesh_ref: list = []
    try:
        return _run(op, comm, nbytes, device, dtype, iters, warmup, mesh_ref)
    finally:
        for m in mesh_ref:
            m.close()


def _run(op: str, comm: Comm, nbytes: int, device, dtype, iters: int, warmup: int, mesh_ref: list) -> float:
    W = comm.world
    esz = torch.tensor([], dtype=dtype).element_size()
    n = max(W, nbytes // esz // W * W)
    if op == "all_gather":
        inp = torch.randn(n // W, device=device).to(dtype)
        out = torch.empty(n, device=device, dtype=dtype)
        fn = lambda: comm.all_gather(out, inp, async_op=False)  # noqa: E731
    elif op == "ipc_mesh_all_gather":
        # device-driven pull from every peer's symmetric heap (parallel/xgmi_mesh.py); GPU only. bench.py runs the
        # mesh rows in a child process after its result line is out (a new transport never risks the number)
        from ..parallel.xgmi_mesh import XgmiMesh
        m = n // W * esz
        mesh = XgmiMesh(comm, device, {"p16": (m, 1)})
        mesh_ref.append(mesh)
        shard = mesh.region_tensor("p16", dtype, n // W)
        shard.copy_(torch.randn(n // W, device=device).to(dtype))
        out = torch.empty(n, device=device, dtype=dtype)
        fn = lambda: (mesh.all_gather_pull(out, shard), DONE)[1]  # noqa: E731
    elif op == "ipc_mesh_reduce_scatter":
        from ..parallel.xgmi_mesh import XgmiMesh, rs_region_bytes
        mesh = XgmiMesh(comm, device, {"rs": (rs_region_bytes(W, n // W), 2)})
        mesh_ref.append(mesh)
        inp = torch.randn(n, device=device).to(dtype)
        out = torch.empty(n // W, device=device, dtype=dtype)
        fn = lambda: (mesh.reduce_scatter(out, inp, 1.0, False), DONE)[1]  # noqa: E731
    elif op == "ipc_mesh_all_to_all":
        # the EP token exchange (parallel/ep.py MeshExpertDispatcher) with balanced routing: E = 2W experts, every
        # expert gets the same number of 4096-wide rows, one dispatch = device count exchange + push + copy-out
        from ..parallel.ep import MeshExpertDispatcher
        D, E = 4096, 2 * W
        rows = max(E, n // D // E * E)
        disp = MeshExpertDispatcher(comm, E, device, rows, D, dtype, capacity_factor=1.0)
        mesh_ref.append(disp.mesh)
        x = torch.randn(rows, D, device=device).to(dtype)
        offsets = (torch.arange(E + 1, device=device) * (rows // E)).to(torch.int32)
        counts = (offsets[1:] - offsets[:-1]).long()
        fn = lambda: (disp.dispatch(x, counts, offsets), DONE)[1]  # noqa: E731
    elif op == "reduce_scatter":
        inp = torch.randn(n, device=device).to(dtype)
        out = torch.empty(n // W, device=device, dtype=dtype)
        fn = lambda: comm.reduce_scatter(out, inp, avg=False, async_op=False)  # noqa: E731
    elif op == "all_reduce":
        buf = torch.randn(n, device=device).to(dtype)
        fn = lambda: comm.all_reduce(buf, async_op=False)  # noqa: E731
    elif op == "all_to_all":
        inp = torch.randn(n, device=device).to(dtype)
        out = torch.empty(n, device=device, dtype=dtype)
        fn = lambda: comm.all_to_all_single(out, inp)  # noqa: E731
    else:
        raise ValueError(op)
    sync = torch.cuda.synchronize if device.type == "cuda" else (lambda: None)
    for _ in range(warmup):
        fn().wait()
    sync()
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn().wait()
    sync()
    dt = (time.perf_counter() - t0) / iters
    t = torch.tensor([dt], dtype=torch.float32, device=device)
    comm.all_reduce_max(t)  # the slowest rank defines the collective's time
    return float(t)



def sweep(comm: Comm, device,
          ops: Sequence[str] = ("all_gather", "reduce_scatter", "all_reduce", "all_to_all"),
          sizes_mb: Sequence[float] = (16, 64, 256), dtype=torch.bfloat16, iters: int = 5,
          warmup: int = 2) -> List[Dict]:
    rows = []
    for op in ops:
        for mb in sizes_mb:
            nbytes = int(mb * (1 << 20))
            try:
                dt = run(op, comm, nbytes, device, dtype, iters, warmup)
            except Exception as e:  # noqa: BLE001 -- record it; the caller's watchdog covers a rank left behind
                rows.append({"op": op, "MiB": mb, "error": f"{type(e).__name__}: {e}"[:200], "world": comm.world})
                continue
            algbw = nbytes / dt / 1e9
            rows.append({"op": op, "MiB": mb, "time_us": round(dt * 1e6, 1), "algbw_GBps": round(algbw, 1),
                         "busbw_GBps": round(algbw * FACTOR[op](comm.world), 1), "world": comm.world})
    return rows
