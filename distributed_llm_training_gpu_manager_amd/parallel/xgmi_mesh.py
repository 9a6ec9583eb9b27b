"""Device-driven xGMI mesh transport over HIP IPC symmetric heaps (SURVEY.md §5.8 plan item 3; §2.7 C1, C3, C6).

The reference only asks DeepSpeed for bucketed, overlapped partition all-gathers and gradient reduce-scatters
(``/root/reference/ai_engine/deepspeed_launcher.py:133-141``: ``allgather_partitions``, ``reduce_scatter``,
``overlap_comm``) and, through BASELINE config 5, for an expert all-to-all on its 8-GPU preset world
(``deepspeed_launcher.py:393-406``). On an 8-GPU MI355X node every GPU pair has its own xGMI link, so instead of
stepping a ring around one link at a time each rank reads or writes its peers' memory directly, all links at once.

Every rank allocates ONE heap (``ipc_alloc``: uncached device memory, the same layout on every rank), exports its
IPC handle and maps every peer's heap. Kernels in csrc/kernels/xgmi_mesh.hip then move data and signal with flags
in the heaps; each flag is an epoch counter held on the device, so nothing here reads the device from the host and
every operation can be captured in a HIP graph. The memory-model argument (why a flag orders the data it guards
across GPUs) is written at the top of xgmi_mesh.hip.

Operations (``W`` ranks of one communicator):

* ``all_gather_pull(out, shard)`` -- ZeRO parameter gather: the bf16 parameter partition of every rank lives in its
  heap (``param_shard``), so a gather is one kernel that PULLS each rank's shard over that rank's link straight into
  any output tensor (no staging buffer, no result ring: prefetch can keep any number of groups live). Version flags
  order it against the optimizer: ``quiesce`` (every rank finished reading version v) runs before the optimizer
  overwrites the partition, ``publish`` (version v+1) after.
* ``reduce_scatter(out, x, scale, accumulate)`` -- gradient reduction: each rank pushes chunk p of its gradient (fp32
  cast to bf16 on the fly, or bf16) into slot ``rank`` of rank p's reduce-scatter region, then every rank sums its W
  slots in fp32 in rank order and writes ``out (+)= sum * scale`` (the engine's accumulate fused in).
* EP dispatch / combine (parallel/ep.py ``MeshExpertDispatcher``): routing counts exchanged through the heaps,
  destination offsets computed on the device, rows pushed straight into the owners' buffers in local-expert-major
  order (no regroup copy) and back.

Each channel's region has ``slots`` slots used round-robin by epoch; a producer waits (on the device) until the
consumer acknowledged epoch e - slots before it rewrites slot e % slots. Every wait is bounded (``timeout_s``): a
peer that died leaves a sticky error that ``check()`` raises, not a hung GPU.

``ranks sharing one GPU`` (the tests, gloo for the handle exchange) is supported: the waiting kernels are single
workgroups and the data-moving kernels never wait.
"""
from __future__ import annotations

import math
import threading
import weakref
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .._native import hip_ops
from .comm import Comm, Handle
from ..utils.streams import owned_stream

CNT, DATA, ACK, VER, RDONE = 0, 1, 2, 3, 4
ST_EPOCH, ST_VER, ST_ERR, ST_OVF, ST_SHADOW = 0, 16, 17, 18, 19
CH_RS, CH_DISPATCH, CH_COMBINE = 0, 1, 2
ALIGN = 4096
ALLOC_MODES = ("uncached", "fine-grained", "coarse-grained")


@dataclass
class Region:
    name: str
    slot_bytes: int
    slots: int
    offset: int = 0

    @property
    def nbytes(self) -> int:
        return self.slot_bytes * self.slots


def _round(x: int, m: int = ALIGN) -> int:
    return (int(x) + m - 1) // m * m


# Heaps are kept for the life of the process and handed to the next mesh of the same device and memory kind: an
# uncached heap is never returned to the driver. Freeing one and letting the caching allocator map the memory again
# made later, unrelated engines compute different bits (round 6: synchronous shadow runs after mesh runs in one
# process diverged from the first run in 2-30 of 35 repetitions, and a gather faulted after empty_cache; kept heaps,
# fine-grained or plain heaps: 0 -- tools/diag/r06_stress.sh, README "Determinism"). Shadow meshes only (one process
# builds many of them: the tests, the shadow-rank tools): a heap a peer process maps is exported over IPC, and a job
# builds one mesh per communicator and frees it at exit.
_HEAP_POOL: Dict[Tuple[int, int], List[torch.Tensor]] = {}
_HEAP_LOCK = threading.Lock()


def _pool_take(dev: int, mode: int, nbytes: int) -> Optional[torch.Tensor]:
    with _HEAP_LOCK:
        free = _HEAP_POOL.get((dev, mode), [])
        fit = [i for i, h in enumerate(free) if h.numel() >= nbytes]
        if not fit:
            return None
        # by index: list.remove would compare tensors with ==
        return free.pop(min(fit, key=lambda i: free[i].numel()))


def _pool_give(dev: int, mode: int, heap: torch.Tensor) -> None:
    with _HEAP_LOCK:
        _HEAP_POOL.setdefault((dev, mode), []).append(heap)


def _release_heap(dev: int, mode: int, heap: torch.Tensor) -> None:
    """weakref.finalize of a shadow mesh: its heap goes back to the pool."""
    _pool_give(dev, mode, heap)


class XgmiMesh:
    """Symmetric heap of one communicator plus its device-driven collectives.

    regions: {name: (bytes per slot, slots)} -- identical on every rank (checked). The heap is
    ``[flags][region 0][region 1]...`` with 4 KiB-aligned regions.
    """

    def __init__(self, comm: Comm, device: torch.device, regions: Dict[str, Tuple[int, int]],
                 timeout_s: float = 60.0, alloc_mode: str = "auto"):
        assert device.type == "cuda", "the xGMI mesh needs GPU memory"
        self.comm, self.device = comm, device
        self.W, self.rank = comm.world, comm.rank
        # shadow rank (ShadowComm: rank r of a world-W job alone on this GPU): every "peer" heap is this rank's own
        # and the kernels write peer t's flags / slots as if they were rank t (csrc/kernels/xgmi_mesh.hip) --
        # true-size traffic and the same stream ordering, no IPC. Its collectives run on the mesh streams after a
        # `delay_cycles` spin (async_mode) or inline on the caller's stream (sync), like ShadowComm's.
        self.shadow = getattr(comm, "backend", "") == "shadow"
        self.inline = self.shadow and not getattr(comm, "async_mode", False)
        self.delay_cycles = int(getattr(comm, "delay_cycles", 0)) if self.shadow else 0
        ops = hip_ops()
        off = _round(int(ops.mesh_flag_bytes()))
        self.regions: Dict[str, Region] = {}
        for name, (sb, ns) in regions.items():
            r = Region(name, _round(max(int(sb), 16)), max(1, int(ns)), off)
            self.regions[name] = r
            off += r.nbytes
        self.heap_bytes = off
        layouts: List[Optional[list]] = [None] * self.W
        mine = [(r.name, r.slot_bytes, r.slots, r.offset) for r in self.regions.values()]
        if self.W > 1 and not self.shadow:
            dist.all_gather_object(layouts, mine, group=comm.group)
            assert all(x == mine for x in layouts), f"mesh: heap layouts differ across ranks: {layouts}"
        self.heap, self.alloc_mode = self._alloc(ops, alloc_mode)
        if self.shadow:
            weakref.finalize(self, _release_heap, self._dev_index(), ALLOC_MODES.index(self.alloc_mode), self.heap)
        self._opened: List[int] = []
        ptrs = [0] * self.W
        ptrs[self.rank] = int(self.heap.data_ptr())
        if self.shadow:
            ptrs = [int(self.heap.data_ptr())] * self.W
        elif self.W > 1:
            handles: List[Optional[list]] = [None] * self.W
            dist.all_gather_object(handles, ops.ipc_handle(self.heap).tolist(), group=comm.group)
            with torch.cuda.device(device):
                for r in range(self.W):
                    if r != self.rank:
                        p = int(ops.ipc_open(torch.tensor(handles[r], dtype=torch.uint8)))
                        self._opened.append(p)
                        ptrs[r] = p
        self.peers = torch.tensor(ptrs, dtype=torch.int64, device=device)
        self.state = torch.zeros(int(ops.mesh_state_words()), dtype=torch.int64, device=device)
        # per-channel epoch / counter words, updated by device-side atomics from the mesh's several streams: ordered
        # by the protocol in xgmi_mesh.hip, not by stream edges (the stream audit leaves them to that protocol)
        from ..utils.stream_audit import protocol_memory
        protocol_memory(self.state, "xGMI mesh state words (device atomics, one word set per channel)")
        if self.shadow:
            self.state[ST_SHADOW] = 1
        self.timeout_ticks = int(timeout_s * 100e6)  # s_memrealtime runs at 100 MHz on MI355X
        # one stream per traffic class (parameter gathers / gradient reductions), like the engine's two RCCL
        # communicators: a prefetch gather and a reduce-scatter run concurrently
        self._streams: Dict[str, torch.cuda.Stream] = {k: owned_stream(device, f"mesh-{k}", owner=self) for k in ("ag", "rs")}
        self.closed = False
        self.issued = 0
        if self.W > 1 and not self.shadow:  # nobody may write into a heap before every rank mapped every heap
            self.host_barrier()

    # ------------------------------------------------------------------ setup
    def _dev_index(self) -> int:
        return self.device.index if self.device.index is not None else torch.cuda.current_device()

    def _alloc(self, ops, mode: str):
        """Uncached heap if the driver exports it over IPC; else fine-grained, else plain (recorded). A shadow mesh
        reuses a pooled heap of the kind (a dead shadow mesh's, at least this large), zeroed, when there is one."""
        order = {"auto": (0, 1, 2), "uncached": (0,), "fine-grained": (1,), "coarse-grained": (2,)}[mode]
        err = None
        with torch.cuda.device(self.device):
            for m in order:
                pooled = _pool_take(self._dev_index(), m, self.heap_bytes) if self.shadow else None
                if pooled is not None:
                    torch.cuda.synchronize(self.device)  # the previous owner's kernels are done with it
                    pooled[:self.heap_bytes].zero_()
                    torch.cuda.synchronize(self.device)
                    return pooled, ALLOC_MODES[m]
                try:
                    buf = ops.ipc_alloc(self.heap_bytes, m)
                    if self.W > 1 and not self.shadow:
                        ops.ipc_handle(buf)  # exportable?
                    return buf, ALLOC_MODES[m]
                except RuntimeError as e:  # try the next memory kind
                    err = e
        raise RuntimeError(f"xGMI mesh: no exportable heap of {self.heap_bytes} bytes: {err}")

    def host_barrier(self) -> None:
        torch.cuda.synchronize(self.device)
        if self.W > 1 and not self.shadow:
            if self.comm.backend == "nccl":
                t = torch.zeros(1, device=self.device)
                dist.all_reduce(t, group=self.comm.group)
                torch.cuda.synchronize(self.device)
            else:
                dist.barrier(group=self.comm.group)

    def region_tensor(self, name: str, dtype: torch.dtype, numel: int, slot: int = 0) -> torch.Tensor:
        r = self.regions[name]
        esz = torch.tensor([], dtype=dtype).element_size()
        assert numel * esz <= r.slot_bytes, f"region {name}: {numel} x {esz} B does not fit {r.slot_bytes} B"
        o = r.offset + slot * r.slot_bytes
        return self.heap[o:o + numel * esz].view(dtype)

    def offset_of(self, t: torch.Tensor) -> int:
        """Byte offset of tensor storage `t` inside this rank's heap (it must live there)."""
        off = int(t.data_ptr()) - int(self.heap.data_ptr())
        assert 0 <= off and off + t.numel() * t.element_size() <= self.heap_bytes, "tensor is not in the mesh heap"
        return off

    # ------------------------------------------------------------------ primitives
    def _sync(self, ch: int, inc: int, val: int, store_kind: int, wait_kind: int, lag: int = 0) -> None:
        hip_ops().mesh_sync(self.state, self.peers, self.rank, ch, inc, val, store_kind, wait_kind, lag,
                            self.timeout_ticks)

    def begin(self, ch: int, slots: int) -> None:
        """Open the next epoch of channel `ch`: wait until every rank released slot (e % slots)."""
        self._sync(ch, ST_EPOCH + ch, ST_EPOCH + ch, -1, ACK, slots)

    def wait_data(self, ch: int) -> None:
        self._sync(ch, -1, ST_EPOCH + ch, -1, DATA, 0)

    def publish(self) -> None:
        """This rank's parameter partition is final for the next version (after the optimizer wrote it)."""
        self._sync(0, ST_VER, ST_VER, VER, -1)

    def wait_version(self) -> None:
        self._sync(0, -1, ST_VER, -1, VER, 0)

    def quiesce(self) -> None:
        """Every rank finished reading the current version of the partitions (before overwriting its own)."""
        self._sync(0, -1, ST_VER, RDONE, RDONE, 0)

    def stream(self, key: str = "ag") -> torch.cuda.Stream:
        return self._streams[key]

    def run_async(self, fn: Callable[[], None], tensors: Sequence[torch.Tensor], key: str = "ag") -> Handle:
        """Run `fn` on the mesh stream after the work queued on the current stream (as RCCL orders a
        collective), keep `tensors` alive for it, and return a Handle whose wait() orders the waiting stream
        after it (no host synchronisation)."""
        if self.inline:  # synchronous shadow rank: on the caller's stream
            fn()
            return Handle()
        cur = torch.cuda.current_stream(self.device)
        s = self.stream(key)
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            if self.delay_cycles:
                torch.cuda._sleep(self.delay_cycles)  # a consumer that forgets to wait reads stale data, every run
            fn()
            ev = torch.cuda.Event()
            ev.record(s)
        for t in tensors:
            if t is not None and t.is_cuda:
                t.record_stream(s)
        self.issued += 1
        dev = self.device
        return Handle(post=lambda: torch.cuda.current_stream(dev).wait_event(ev))

    # ------------------------------------------------------------------ ZeRO collectives
    def all_gather_pull(self, out: torch.Tensor, shard: torch.Tensor) -> None:
        """out = concat over ranks of each rank's `shard` (a tensor inside the heap, the same offset on every rank)."""
        off = self.offset_of(shard)
        assert out.numel() == self.W * shard.numel() and out.dtype == shard.dtype
        self.wait_version()
        hip_ops().mesh_pull(out, self.peers, off, self.heap_bytes)

    def reduce_scatter(self, out: torch.Tensor, x: torch.Tensor, scale: float, accumulate: bool,
                       region: str = "rs", fp32: bool = False) -> None:
        """out (+)= scale * sum over ranks of x[rank's chunk], summed in fp32 in rank order. The chunks travel as bf16
        (rounded on the fly) or, with ``fp32`` (an fp32 `x`: the once-per-step reduce of the local accumulator), as
        fp32: the same sum RCCL's fp32 reduce-scatter computes, up to the order of the fp32 additions."""
        r = self.regions[region]
        rank_stride = r.slot_bytes // self.W // 256 * 256
        args = (self.peers, self.state, self.rank, CH_RS, r.offset, r.slot_bytes, rank_stride, r.slots,
                self.heap_bytes, bool(fp32))
        self.begin(CH_RS, r.slots)
        hip_ops().mesh_rs_push(x.contiguous(), *args)
        self.wait_data(CH_RS)
        hip_ops().mesh_rs_reduce(out, float(scale), bool(accumulate), *args)

    # ------------------------------------------------------------------ health
    def check(self) -> None:
        """Raise if a wait timed out (a peer died or the protocol desynchronised). A host read: call it at a step
        boundary, not inside a captured region."""
        err = int(self.state[ST_ERR])
        if err:
            raise RuntimeError("xGMI mesh: a device-side wait timed out (a peer stopped responding)")

    def overflowed(self) -> bool:
        return bool(int(self.state[ST_OVF]))

    def close(self) -> None:
        """Unmap the peers' heaps, then wait for every rank to have done the same before this rank's heap may be
        freed (an exporter must not free memory a peer still maps). Collective."""
        if self.closed:
            return
        torch.cuda.synchronize(self.device)
        ops = hip_ops()
        for p in self._opened:
            ops.ipc_close(p)
        self._opened = []
        if not self.shadow:
            self.host_barrier()
        self.closed = True


def rs_region_bytes(world: int, max_chunk_elems: int, elem_bytes: int = 2) -> int:
    """Bytes of one reduce-scatter slot: W chunks of the largest shard, 256-byte aligned each."""
    return world * _round(max_chunk_elems * elem_bytes, 256)


def ep_region_bytes(world: int, n_experts: int, rows: int, row_bytes: int) -> Tuple[int, int]:
    """(header bytes, slot bytes) of an EP region holding `rows` rows: the [W, E] int32 count header, then rows."""
    hdr = _round(world * n_experts * 4, 256)
    return hdr, hdr + rows * row_bytes


def capacity_rows(tokens_k: int, world: int, factor: Optional[float]) -> int:
    """Receive rows of an EP rank. factor None = dropless: the worst case, every row of every source (W x
    tokens_k) -- on a 288 GB MI355X the slot costs little (Mixtral EP = 8, seq 4096, top-2: 65,536 rows x 8 KiB =
    512 MiB). A factor gives a static capacity of factor x the balanced share (each rank receives tokens_k rows on
    average under balanced routing), at most the worst case. 64-row aligned."""
    worst = world * tokens_k
    c = worst if factor is None else min(int(math.ceil(factor * tokens_k)), worst)
    return max(64, (c + 63) // 64 * 64)
