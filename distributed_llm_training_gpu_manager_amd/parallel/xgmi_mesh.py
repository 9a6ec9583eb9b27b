"""Peer-write xGMI mesh all-gather (plan item 3) over HIP IPC symmetric buffers.

The reference only asks DeepSpeed for bucketed, overlapped partition all-gathers
(``/root/reference/ai_engine/deepspeed_launcher.py:133-141``: ``allgather_partitions``,
``allgather_bucket_size``, ``overlap_comm``); this is the MI355X-native transport option for them.

Every rank allocates one symmetric buffer (``cap`` bytes, its own hipMalloc), exports its IPC handle, and maps
every peer's buffer (``hipIpcOpenMemHandle``; on one 8-GPU MI355X node every pair of GPUs has its own xGMI link).
An all-gather is then:

    entry barrier              peers are done reading the previous result out of the buffers
    own shard -> own slot      local copy
    mesh_push                  ONE kernel writes this rank's shard into slot `rank` of all W-1 peers' buffers
                               (16-byte vector stores over xGMI, all links at once; csrc/kernels/xgmi_mesh.hip)
    exit barrier               every peer's push has completed -> every slot of this rank's buffer is written

The barriers are stream-ordered on RCCL (a 1-element all-reduce behind the push kernel on the compute stream), so
the sequence needs no host synchronisation; on gloo (tests: several ranks sharing one GPU) they are a device
synchronise + ``dist.barrier``. The gathered result is a view of the symmetric buffer, valid until the next
gather. Compared with RCCL's ring all-gather this moves each shard once per link with no intermediate hops;
``utils/commbench.py`` measures both (``bench.py`` runs that sweep on the multi-GPU node after its timed steps).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from .._native import hip_ops
from .comm import Comm


class XgmiMesh:
    def __init__(self, comm: Comm, cap_bytes: int, device: torch.device):
        assert device.type == "cuda", "the xGMI mesh needs GPU buffers"
        self.comm, self.device = comm, device
        self.cap = (int(cap_bytes) + 15) // 16 * 16
        ops = hip_ops()
        with torch.cuda.device(device):
            self.buf = ops.ipc_alloc(self.cap)
        handle = ops.ipc_handle(self.buf).tolist()
        handles: List[Optional[list]] = [None] * comm.world
        dist.all_gather_object(handles, handle, group=comm.group)
        self._opened: List[int] = []
        ptrs = []
        with torch.cuda.device(device):
            for r in range(comm.world):
                if r == comm.rank:
                    continue
                p = int(ops.ipc_open(torch.tensor(handles[r], dtype=torch.uint8)))
                self._opened.append(p)
                ptrs.append(p)
        self.peers = torch.tensor(ptrs, dtype=torch.int64, device=device)
        self._nccl = comm.backend == "nccl"
        self._flag = torch.zeros(1, device=device)

    def _barrier(self) -> None:
        if self.comm.world == 1:
            return
        if self._nccl:  # stream-ordered: RCCL's kernel runs after everything queued before it on this stream
            dist.all_reduce(self._flag, group=self.comm.group)
        else:
            torch.cuda.synchronize(self.device)
            dist.barrier(group=self.comm.group)

    def all_gather(self, shard: torch.Tensor) -> torch.Tensor:
        """Gather `shard` (same size on every rank, 16-byte multiple) from all ranks; returns a view of the
        symmetric buffer [world * shard.numel()] in shard's dtype, rank-major."""
        shard = shard.contiguous()
        nb = shard.numel() * shard.element_size()
        W, r = self.comm.world, self.comm.rank
        assert nb % 16 == 0 and W * nb <= self.cap, "mesh all-gather: shard must be 16-byte sized and fit the buffer"
        self._barrier()  # every peer is done with the previous contents
        self.buf[r * nb:(r + 1) * nb].copy_(shard.view(torch.uint8).view(-1))
        hip_ops().mesh_push(shard, self.peers, r * nb, self.cap)
        self._barrier()  # every peer's push into this buffer has completed
        return self.buf[:W * nb].view(shard.dtype)

    def close(self) -> None:
        """Unmap the peers' buffers, then wait for every rank to have done the same before this rank's own
        buffer may be freed (an exporter must not free memory a peer still maps). Collective."""
        if self._opened:
            torch.cuda.synchronize(self.device)
            ops = hip_ops()
            for p in self._opened:
                ops.ipc_close(p)
            self._opened = []
        if self.comm.world > 1:
            torch.cuda.synchronize(self.device)
            dist.barrier(group=self.comm.group)
