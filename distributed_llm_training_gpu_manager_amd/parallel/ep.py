"""Expert parallelism: process groups and the token all-to-all (BASELINE config 5).

Layout: ``world = ep_size x expert_dp``. EP groups are contiguous rank blocks
(``[0..ep-1], [ep..2ep-1], ...``) -- on one 8-GPU MI355X node with ep=8 the
all-to-all runs over the full xGMI mesh, where every GPU pair has a direct link,
which is exactly the traffic pattern a point-to-point fabric serves best (no
ring). Expert-data-parallel groups hold the same experts (rank i, i+ep, ...) and
carry the ZeRO partitioning of the expert weights.

The dispatcher moves permuted token rows to the ranks that own their experts and
back with ``all_to_all_single`` and uneven splits. The split sizes are exchanged
first (one tiny all-to-all of the [W, El] count matrix) and read on the host ONCE per
MoE layer and micro-batch -- the send and receive counts in a single device-to-host
copy, because RCCL's uneven all-to-all takes its split sizes on the host; the
backward reuses the forward's splits (no exchange, no read). The permutation from the
received [source rank][local expert] order to local-expert-major order is built on the
device (``_regroup_index``), never as a host list.

:class:`MeshExpertDispatcher` is the MI355X-native transport (parallel/xgmi_mesh.py): the routing counts travel
through the ranks' symmetric heaps, every destination offset is computed on the device, each rank writes its rows
straight into the expert owners' receive buffers over xGMI in local-expert-major order (no regroup copy), and the
combine is the mirror image. The exchange is DROPLESS by default: every rank's receive slot holds the worst case
(all W x T x k rows of the EP group), so no routing can overflow it (Mixtral-8x7B EP = 8, seq 4096, top-2: 512 MiB
per slot of a 288 GB MI355X). The rows handed to the expert GEMMs are either a static worst-case tensor (no host read
at all: the EP micro-batch loop can be captured in a HIP graph; chosen when those activations fit the HBM plan) or,
``sized_output``, exactly the received rows (one host read of the received count per dispatch, like the RCCL path's
split exchange). An explicit ``capacity_factor`` gives the old static capacity (capturable with less memory); a
routing that overflows it raises at the next step boundary (:meth:`MeshExpertDispatcher.overflowed`, read by
``ZeroEngine.check_transport``) instead of training on dropped tokens. The RCCL dispatcher above stays the default
transport and the fallback (``EngineConfig.xgmi_mesh``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

from .comm import Comm


def build_ep_comms(ep_size: int, comm: Optional[Comm] = None) -> Tuple[Optional[Comm], Optional[Comm]]:
    """Return (ep_comm, expert_dp_comm) for this rank; every rank must call this collectively.

    The EP all-to-all always gets a communicator of its own -- also when ep_size == world -- so the
    token exchange runs on its own RCCL stream instead of queueing behind the dense gradient
    reduce-scatters on the world communicator."""
    comm = comm or Comm()
    if comm.world == 1:
        return None, None
    world, rank = comm.world, comm.rank
    assert world % ep_size == 0, "world size must be a multiple of expert_parallel_size"
    ep_comm = edp_comm = None
    for b in range(world // ep_size):
        ranks = list(range(b * ep_size, (b + 1) * ep_size))
        g = comm.duplicate() if ep_size == world else comm.new_group(ranks)
        if rank in ranks:
            ep_comm = g
    dp = world // ep_size
    for i in range(ep_size):
        ranks = list(range(i, world, ep_size))
        g = comm.new_group(ranks)
        if rank in ranks:
            edp_comm = g
    return ep_comm, edp_comm


@dataclass
class DispatchCtx:
    send_splits: List[int]
    recv_splits: List[int]
    regroup: Optional[torch.Tensor]  # recv order -> local-expert-major order
    local_counts: Optional[List[int]]  # host copy (None until asked for at EP = 1)
    local_offsets: Optional[torch.Tensor] = None  # int32 [El + 1] on the device: expert row ranges
    nrows: Optional[torch.Tensor] = None  # int32 [1] on the device: valid rows of a capacity-sized dispatch output
    plan: Optional[torch.Tensor] = None  # mesh transfer tables (MeshExpertDispatcher)
    out_rows: int = 0  # rows of the mesh dispatch output (>= the valid rows)

    def counts(self) -> List[int]:
        """Host per-local-expert row counts (a device sync at EP = 1; the per-expert fallback path only)."""
        if self.local_counts is None:
            o = self.local_offsets.tolist()
            self.local_counts = [b - a for a, b in zip(o[:-1], o[1:])]
        return self.local_counts


def _regroup_index(mat: torch.Tensor, total: int) -> torch.Tensor:
    """Device permutation of the received rows, [source rank][local expert] order -> [local expert][source
    rank] order: entry j of the output is the received row that goes to position j. mat [W, El] counts (on the
    device); `total` = mat.sum() (known on the host). No host list, no host-to-device copy of indices."""
    W, El = mat.shape
    dev = mat.device
    if total == 0:
        return torch.zeros(0, dtype=torch.long, device=dev)
    m = mat.to(torch.long)
    src_start = (m.reshape(-1).cumsum(0) - m.reshape(-1)).view(W, El)  # block (s, e) in received order
    mt = m.t().reshape(-1)  # blocks in output order (e, s)
    dst_start = mt.cumsum(0) - mt
    shift = src_start.t().reshape(-1) - dst_start  # received position - output position, per block
    return torch.arange(total, device=dev) + torch.repeat_interleave(shift, mt, output_size=total)


class ExpertDispatcher:
    def __init__(self, ep_comm: Optional[Comm], n_experts: int):
        self.comm = ep_comm
        self.W = ep_comm.world if ep_comm is not None else 1
        self.rank = ep_comm.rank if ep_comm is not None else 0
        self.E = n_experts
        assert n_experts % self.W == 0, "n_experts must be divisible by the EP size"
        self.El = n_experts // self.W

    def dispatch(self, x_sorted: torch.Tensor, counts: torch.Tensor,
                 offsets: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, DispatchCtx]:
        """x_sorted: rows grouped by global expert id (counts[e] rows each; `offsets` = the int32 exclusive
        prefix of counts on the device, from ops.moe_permute). At EP = 1 nothing is read on the host."""
        if self.W == 1:
            if offsets is None:
                offsets = torch.zeros(self.E + 1, dtype=torch.int32, device=counts.device)
                offsets[1:] = torch.cumsum(counts, 0)
            return x_sorted, DispatchCtx([x_sorted.shape[0]], [x_sorted.shape[0]], None, None, offsets)
        recv = torch.empty_like(counts)
        self.comm.all_to_all_single(recv, counts.contiguous())  # [src, local expert] counts
        # the only host read of the layer: send counts and received [src, local expert] counts in one copy
        both = torch.cat([counts.reshape(-1), recv.reshape(-1)]).to(torch.int64).cpu()
        mat = both[self.E:].view(self.W, self.El)
        c_send = both[:self.E].view(self.W, self.El).sum(1).tolist()
        c_recv = mat.sum(1).tolist()
        out = x_sorted.new_empty((sum(c_recv), x_sorted.shape[1]))
        self.comm.all_to_all_single(out, x_sorted.contiguous(), c_recv, c_send)
        regroup = _regroup_index(recv.view(self.W, self.El), sum(c_recv))
        lc = mat.sum(0).tolist()
        lo = torch.zeros(self.El + 1, dtype=torch.int32, device=x_sorted.device)
        lo[1:] = recv.view(self.W, self.El).sum(0).cumsum(0)
        ctx = DispatchCtx(c_send, c_recv, regroup, lc, lo)
        return out.index_select(0, regroup), ctx

    def redispatch(self, rows_sorted: torch.Tensor, ctx: DispatchCtx) -> torch.Tensor:
        """Send another [N, D] tensor laid out like the dispatched rows (backward: d outputs)."""
        if self.W == 1:
            return rows_sorted
        out = rows_sorted.new_empty((sum(ctx.recv_splits), rows_sorted.shape[1]))
        self.comm.all_to_all_single(out, rows_sorted.contiguous(), ctx.recv_splits, ctx.send_splits)
        return out.index_select(0, ctx.regroup)

    def combine(self, y_local: torch.Tensor, ctx: DispatchCtx) -> torch.Tensor:
        """Inverse of dispatch: local-expert-major rows back to the source ranks, expert-sorted order."""
        if self.W == 1:
            return y_local
        y_recv = torch.empty_like(y_local)
        y_recv.index_copy_(0, ctx.regroup, y_local)
        out = y_local.new_empty((sum(ctx.send_splits), y_local.shape[1]))
        self.comm.all_to_all_single(out, y_recv, ctx.send_splits, ctx.recv_splits)
        return out


class MeshExpertDispatcher:
    """EP token exchange over the xGMI mesh (csrc/kernels/xgmi_mesh.hip), device-driven end to end.

    dispatch:   mesh_ep_plan (epoch open + count exchange + tables, one workgroup) -> mesh_push_rows (this rank's
                expert-sorted rows into every owner's slot at device-computed rows) -> wait -> copy-out of the
                local-expert-major rows (ACKs the slot)
    combine:    epoch open -> push each (local expert, source) block back to the source's expert-sorted rows -> wait
                -> copy-out of the [tokens x k, D] rows
    redispatch: the dispatch pattern again with the forward's tables (backward: d outputs)

    capacity_factor None (dropless): the receive slot holds W x rows, so the device tables never clamp a row.
    The dispatch output then has ``C`` rows (static: capturable) or, with ``sized_output``, the received count
    rounded up to 64 (one host read per dispatch). ``ctx.local_offsets`` / ``ctx.nrows`` say which rows are valid;
    every consumer (grouped GEMMs, SwiGLU, the combine push) reads only those.
    """

    def __init__(self, ep_comm: Comm, n_experts: int, device: torch.device, rows: int, d_model: int,
                 dtype: torch.dtype, capacity_factor: Optional[float] = None, slots: int = 2, timeout_s: float = 60.0,
                 sized_output: bool = False):
        from .._native import hip_ops
        from .xgmi_mesh import CH_COMBINE, CH_DISPATCH, XgmiMesh, capacity_rows, ep_region_bytes
        self.W, self.rank, self.E = ep_comm.world, ep_comm.rank, n_experts
        assert n_experts % self.W == 0, "n_experts must be divisible by the EP size"
        self.El = n_experts // self.W
        self.rows, self.D, self.dtype = int(rows), int(d_model), dtype
        self.dropless = capacity_factor is None
        self.sized = bool(sized_output) and self.dropless
        esz = torch.tensor([], dtype=dtype).element_size()
        self.C = capacity_rows(self.rows, self.W, capacity_factor)
        self.hdr, disp = ep_region_bytes(self.W, n_experts, self.C, d_model * esz)
        self.mesh = XgmiMesh(ep_comm, device, {"ep_dispatch": (disp, slots), "ep_combine": (self.rows * d_model * esz,
                                                                                          slots)}, timeout_s)
        self.L = list(hip_ops().mesh_plan_layout(self.W, n_experts))
        self._A, self._B = self.mesh.regions["ep_dispatch"], self.mesh.regions["ep_combine"]
        self._cd, self._cc = CH_DISPATCH, CH_COMBINE
        self.max_rows_seen = 0  # sized_output: the largest received count so far (host-side record)

    def _push(self, x: torch.Tensor, plan: torch.Tensor, combine: bool) -> None:
        from .._native import hip_ops
        m, r = self.mesh, (self._B if combine else self._A)
        hip_ops().mesh_push_rows(x.contiguous(), plan, combine, m.peers, m.state, m.rank,
                                 self._cc if combine else self._cd, r.offset, r.slot_bytes,
                                 0 if combine else self.hdr, r.slots, self.rows if combine else self.C,
                                 m.heap_bytes, self.E)

    def _copy(self, out: torch.Tensor, nrows: Optional[torch.Tensor], combine: bool) -> None:
        from .._native import hip_ops
        m, r = self.mesh, (self._B if combine else self._A)
        hip_ops().mesh_copy_rows(out, nrows, m.peers, m.state, m.rank, self._cc if combine else self._cd,
                                 r.offset, r.slot_bytes, 0 if combine else self.hdr, r.slots, m.heap_bytes)

    def dispatch(self, x_sorted: torch.Tensor, counts: torch.Tensor,
                 offsets: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, DispatchCtx]:
        from .._native import hip_ops
        assert x_sorted.shape == (self.rows, self.D) and x_sorted.dtype == self.dtype, \
            f"mesh dispatch sized for [{self.rows}, {self.D}] {self.dtype} rows, got {tuple(x_sorted.shape)}"
        if offsets is None:
            offsets = torch.zeros(self.E + 1, dtype=torch.int32, device=counts.device)
            offsets[1:] = torch.cumsum(counts, 0)
        m, A = self.mesh, self._A
        plan = torch.empty(self.L[-1], dtype=torch.int32, device=x_sorted.device)
        hip_ops().mesh_ep_plan(offsets.contiguous(), plan, self.C, m.peers, m.state, m.rank, self._cd, A.offset,
                               A.slot_bytes, A.slots, m.heap_bytes, m.timeout_ticks)
        self._push(x_sorted, plan, False)
        m.wait_data(self._cd)
        nrows = plan[self.L[0]:self.L[0] + 1]
        out_rows = self.C
        if self.sized:  # the received count on the host (the plan kernel has it after the count exchange)
            n = int(nrows)
            self.max_rows_seen = max(self.max_rows_seen, n)
            out_rows = max(64, (n + 63) // 64 * 64)
        out = x_sorted.new_empty((out_rows, self.D))
        self._copy(out, nrows, False)
        lo = self.L[3]
        ctx = DispatchCtx([], [], None, None, plan[lo:lo + self.El + 1], nrows=nrows, plan=plan, out_rows=out_rows)
        return out, ctx

    def redispatch(self, rows_sorted: torch.Tensor, ctx: DispatchCtx) -> torch.Tensor:
        assert rows_sorted.shape == (self.rows, self.D)
        self.mesh.begin(self._cd, self._A.slots)
        self._push(rows_sorted, ctx.plan, False)
        self.mesh.wait_data(self._cd)
        out = rows_sorted.new_empty((ctx.out_rows, self.D))
        self._copy(out, ctx.nrows, False)
        return out

    def combine(self, y_local: torch.Tensor, ctx: DispatchCtx) -> torch.Tensor:
        assert y_local.shape == (ctx.out_rows, self.D)
        self.mesh.begin(self._cc, self._B.slots)
        self._push(y_local, ctx.plan, True)
        self.mesh.wait_data(self._cc)
        out = y_local.new_empty((self.rows, self.D))
        self._copy(out, None, True)
        return out

    def overflowed(self) -> bool:
        """Did any dispatch so far overflow the receive capacity (host read: call at a step boundary)? Never in the
        dropless mode (an assertion); in the capacity mode the engine raises on it."""
        return self.mesh.overflowed()

    def close(self) -> None:
        self.mesh.close()


def static_dispatch_fits(rows_worst: int, d_model: int, ffn_dim: int, n_layers: int, activation_checkpointing: bool,
                         hbm_bytes: float, fraction: float = 0.10, esz: int = 2) -> bool:
    """Dropless mesh EP: can every MoE layer keep worst-case-sized expert activations (x, gate/up, SwiGLU output, y:
    D + 3F + D per row) within `fraction` of HBM? Then the dispatch output is a static tensor and the EP loop stays
    capturable; otherwise it is sized per dispatch by one host read."""
    per_layer = rows_worst * (2 * d_model + 3 * ffn_dim) * esz
    live_layers = 1 if activation_checkpointing else n_layers
    # backward temporaries of one layer (dA, dGU, dX) on top of the saved ones
    return per_layer * live_layers + rows_worst * (3 * ffn_dim + d_model) * esz <= fraction * hbm_bytes
