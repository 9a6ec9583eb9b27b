"""Peer-write mesh all-gather over HIP IPC symmetric buffers (parallel/xgmi_mesh.py, csrc/kernels/xgmi_mesh.hip).

Ranks share one MI355X here (IPC within one device; gloo carries the handle exchange and the barriers -- RCCL
refuses two ranks on one GPU): every rank exports its buffer, maps every peer's, and its push kernel writes its
shard into all peers' buffers. Checked bit-exactly against the concatenation of every rank's shard, over several
consecutive gathers (the entry barrier must keep a push from overwriting a slot a peer is still reading)."""
import os
import socket

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


def _shard(rank, it, n):
    g = torch.Generator().manual_seed(1000 * it + rank)
    return torch.randn(n, generator=g).to(torch.bfloat16)


def _worker(rank, world, port, n, iters, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from distributed_llm_training_gpu_manager_amd.parallel.comm import Comm
    from distributed_llm_training_gpu_manager_amd.parallel.xgmi_mesh import XgmiMesh
    mesh = XgmiMesh(Comm(), world * n * 2, dev)
    ok = True
    for it in range(iters):
        got = mesh.all_gather(_shard(rank, it, n).to(dev)).cpu()
        want = torch.cat([_shard(r, it, n) for r in range(world)])
        ok = ok and torch.equal(got, want)
    mesh.close()
    flag = torch.tensor([1 if ok else 0])
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if rank == 0:
        torch.save({"ok": int(flag)}, out_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 4096), (4, 1 << 20)])
def test_ipc_mesh_all_gather_matches_concat(tmp_path, world, n):
    out = str(tmp_path / "mesh.pt")
    mp.spawn(_worker, args=(world, _free_port(), n, 3, out), nprocs=world, join=True)
    assert torch.load(out, weights_only=True)["ok"] == 1
