"""Unit abstraction shared by every model family.

A model is a sequence of *units* (embedding, N transformer blocks, head). Each
unit declares its parameters (:class:`ParamSpec`) and implements an explicit
``forward`` / ``backward`` pair over plain tensors:

* the ZeRO engine owns all parameter storage as flat buffers (one flat segment
  per unit) and hands the unit *views* of the gathered/persistent bf16 buffer;
* ``backward`` writes parameter gradients directly into views of a flat bf16
  gradient buffer (GEMMs use ``out=`` so no extra copies), which the engine then
  reduce-scatters / accumulates -- this is the MI355X replacement for DeepSpeed's
  module hooks + contiguous gradient buffer;
* nothing in the hot path uses torch.autograd: activation lifetime and memory are
  explicit, which is what lets the 288 GB HBM plan drop activation recompute.

:class:`AutogradUnit` adapts a plain PyTorch forward for families whose
backward is not hand-written (it recomputes the forward under autograd in
backward, i.e. activation checkpointing at unit granularity).
"""
from __future__ import annotations

import math
import zlib
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch

Params = Dict[str, torch.Tensor]


@dataclass
class ParamSpec:
    name: str
    shape: Tuple[int, ...]
    init: str = "normal"  # normal | ones | zeros | normal_scaled
    std: float = 0.02
    weight_decay: bool = True
    experts: int = 0  # >0: leading dim indexes experts; each expert is seeded by its GLOBAL index
    expert_offset: int = 0
    tcache: bool = False  # 2-D weight whose transpose the engine may cache (fast dX GEMM layout)

    @property
    def numel(self) -> int:
        return int(math.prod(self.shape))


@dataclass
class StepContext:
    """Per-micro-batch state shared by all units of one forward/backward."""
    batch: int
    seq_len: int
    input_ids: torch.Tensor  # [B, S] int64
    labels: torch.Tensor  # [B, S] int64
    grad_scale: float  # d(loss_total)/d(loss_row)
    rope: Optional[Tuple[torch.Tensor, torch.Tensor]] = None
    ep_group: Any = None
    sp_group: Any = None  # sequence-parallel Comm (parallel/sp.py): seq_len is then the LOCAL chunk
    aux: Dict[str, Any] = field(default_factory=dict)
    grad_acc: bool = False  # backward ADDS into the gradient views (later micro-batch / tied second visit)
    micro_index: int = 0  # position of this micro-batch in the optimizer step
    last_micro: bool = True
    # units may keep weight-gradient operands across the step's micro-batches and run ONE GEMM with the
    # micro-batches concatenated along K at the last one (their gradients go straight to fp32 targets)
    defer_wgrad: bool = False
    # last micro-batch, single rank: fp32 [2] the units add [sum g^2, #non-finite] of each expert weight's FINAL
    # gradient to (fused into its dW GEMM), counting the weights in aux["expert_stats_weights"]
    expert_stats: Optional[torch.Tensor] = None
    # fp16 path: the dynamic loss scale as a device word (multiplied into the loss gradient on the device)
    loss_scale: Optional[torch.Tensor] = None
    # expert-parallel token exchange shared by every MoE layer (parallel/ep.py MeshExpertDispatcher); None: the
    # layer builds the RCCL dispatcher over ep_group
    ep_dispatcher: Any = None

    @property
    def tokens(self) -> int:
        return self.batch * self.seq_len


class Unit:
    """Base class: subclasses define ``specs`` and forward/backward."""

    name: str = "unit"

    def param_specs(self) -> List[ParamSpec]:
        raise NotImplementedError

    def forward(self, p: Params, x: Any, ctx: StepContext) -> Tuple[Any, Any]:
        """Return (output, saved). Output of the last unit is the loss sum (device scalar)."""
        raise NotImplementedError

    def backward(self, p: Params, g: Params, saved: Any, dy: Any, ctx: StepContext) -> Any:
        """Write (``ctx.grad_acc`` False) or add (True) parameter grads into the views ``g``; return d input.

        ``g`` views are bf16 scratch (reduce-scattered per micro-batch) or fp32 slices of the
        gradient partition itself (accumulated in place, see ops.gemm.grad_mm)."""
        raise NotImplementedError

    # Units whose parameters are needed again at a second position (tied weights)
    def flops(self, ctx: StepContext) -> float:
        return 0.0


def init_param(spec: ParamSpec, out: torch.Tensor, gen: torch.Generator, seed: int = 0) -> None:
    """Deterministic init into a float32 tensor `out` (flat view of the unit).

    Expert tensors are initialised expert by expert from a seed of the global expert
    index, so a model sharded over any expert-parallel size starts from the same weights.
    """
    if spec.experts and spec.init not in ("ones", "zeros"):
        for e in range(spec.experts):
            gen.manual_seed(seed * 7919 + (spec.expert_offset + e) * 104729 + zlib.crc32(spec.name.encode()) % 1000)
            out[e].normal_(0.0, spec.std, generator=gen)
        return
    if spec.init == "ones":
        out.fill_(1.0)
    elif spec.init == "zeros":
        out.zero_()
    else:
        out.normal_(0.0, spec.std, generator=gen)


def _store_grad(dst: torch.Tensor, src: torch.Tensor, acc: bool) -> None:
    """dst (+)= src. fp32 targets on the GPU take the HIP accumulate kernel (one pass, bf16 or fp32 source:
    torch's mixed-dtype add runs ~3x slower and the cast-then-add pair costs two passes)."""
    if (dst.is_cuda and dst.dtype == torch.float32 and src.dtype in (torch.bfloat16, torch.float16, torch.float32)
            and dst.is_contiguous() and src.is_contiguous() and dst.data_ptr() % 16 == 0 and src.data_ptr() % 16 == 0):
        from ..ops.optim import accumulate_
        accumulate_(dst, src.reshape(dst.shape), 1.0, 1.0 if acc else 0.0)
    elif acc:
        dst.add_(src.to(dst.dtype))
    else:
        dst.copy_(src)


class AutogradUnit(Unit):
    """Unit whose backward is derived by autograd.

    ``keep_graph = False``: the forward runs without a graph and the backward recomputes it (minimum
    activation memory). ``keep_graph = True``: the forward records the autograd graph, so its saved
    activations (and the gathered parameter views it references) live until the backward, which then
    only runs the backward kernels -- no second forward. The engine's activation checkpointing still
    applies on top: a checkpointed unit is re-run by the engine right before its backward.
    """

    keep_graph = False

    def fwd(self, p: Params, x: Any, ctx: StepContext) -> Any:
        raise NotImplementedError

    @staticmethod
    def _leaves(p: Params, x: Any):
        leaves = {k: v.detach().requires_grad_(True) for k, v in p.items()}
        xin = x.detach().requires_grad_(x.is_floating_point()) if isinstance(x, torch.Tensor) else x
        return leaves, xin

    def forward(self, p: Params, x: Any, ctx: StepContext):
        if self.keep_graph and torch.is_tensor(x):
            leaves, xin = self._leaves(p, x)
            with torch.enable_grad():
                y = self.fwd(leaves, xin, ctx)
            return y.detach(), ("graph", leaves, xin, y)
        with torch.no_grad():
            y = self.fwd(p, x, ctx)
        return y, x

    def backward(self, p: Params, g: Params, saved: Any, dy: Any, ctx: StepContext):
        if isinstance(saved, tuple) and len(saved) == 4 and saved[0] == "graph":
            _, leaves, xin, y = saved
            if dy is None:  # loss unit
                y.backward()
            else:
                y.backward(dy)
        else:
            leaves, xin = self._leaves(p, saved)
            with torch.enable_grad():
                y = self.fwd(leaves, xin, ctx)
                if dy is None:  # loss unit
                    y.backward()
                else:
                    y.backward(dy)
        for k, leaf in leaves.items():
            if leaf.grad is None:
                if not ctx.grad_acc:
                    g[k].zero_()
            else:
                _store_grad(g[k], leaf.grad, ctx.grad_acc)
        if isinstance(xin, torch.Tensor) and xin.requires_grad:
            return xin.grad
        return None
