"""Probe: can two RCCL ranks share one MI355X? (lets a 1-GPU box exercise the real RCCL collectives).

torchrun --nproc-per-node 2 --master-addr 127.0.0.1 tools/probe_rccl_same_gpu.py
Every rank binds cuda:0 and runs reduce_scatter_tensor(AVG), all_gather_into_tensor, all_reduce and
all_to_all_single with uneven splits, checking the results against host arithmetic.
"""
import datetime
import os
import sys

import torch
import torch.distributed as dist


def main() -> int:
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60),
                            device_id=dev)
    n = 1 << 20
    x = torch.full((n * world,), float(rank + 1), device=dev, dtype=torch.bfloat16)
    out = torch.empty(n, device=dev, dtype=torch.bfloat16)
    dist.reduce_scatter_tensor(out, x, op=dist.ReduceOp.AVG)
    exp = sum(range(1, world + 1)) / world
    ok_rs = bool((out.float() - exp).abs().max() < 1e-2)
    g = torch.empty(n * world, device=dev, dtype=torch.bfloat16)
    dist.all_gather_into_tensor(g, torch.full((n,), float(rank), device=dev, dtype=torch.bfloat16))
    ok_ag = all(bool((g[i * n:(i + 1) * n] == i).all()) for i in range(world))
    s = torch.tensor([1.0, float(rank)], device=dev)
    dist.all_reduce(s)
    ok_ar = abs(float(s[0]) - world) < 1e-6
    # uneven all-to-all: rank r sends (p + 1) rows to peer p
    send = torch.cat([torch.full((p + 1, 4), float(rank * 10 + p), device=dev) for p in range(world)])
    recv = torch.empty((world * (rank + 1), 4), device=dev)
    dist.all_to_all_single(recv, send, [rank + 1] * world, [p + 1 for p in range(world)])
    ok_a2a = all(bool((c == s_ * 10 + rank).all()) for s_, c in enumerate(recv.split(rank + 1)))
    torch.cuda.synchronize()
    print(f"rank {rank}: rs={ok_rs} ag={ok_ag} ar={ok_ar} a2a={ok_a2a}", flush=True)
    dist.destroy_process_group()
    return 0 if (ok_rs and ok_ag and ok_ar and ok_a2a) else 1


if __name__ == "__main__":
    sys.exit(main())
