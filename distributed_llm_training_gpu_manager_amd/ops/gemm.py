"""Weight-gradient GEMM helper: write or accumulate dW straight into the engine's gradient storage.

On MI355X the gradient partition is fp32 and hipBLASLt runs bf16 x bf16 -> fp32 GEMMs
(``aten::mm.dtype_out`` / ``aten::addmm.dtype_out``) at the speed of the bf16-output
GEMM, so micro-batch gradients are accumulated inside the GEMM epilogue (beta = 1)
instead of being rounded to bf16 and added by a separate pass.
"""
from __future__ import annotations

import json
import os
from pathlib import Path
from typing import Optional

import torch

from .._native import hip_available, hip_ops, use_native


# hipBLASLt on gfx950, bf16 x bf16 -> fp32 (measured, tools/probe_dw_layout2.py): both operands with
# the reduction (token) dim strided ("NN", what dW = dy^T x is) ~1.0 PF; one operand K-contiguous
# ~1.27 PF; both ~1.35 PF. The HIP transpose streams at ~4.5 TB/s.
TUNED_DIR = Path(__file__).resolve().parent.parent / "tuned"

_PF = {"NN": 1.0e15, "A": 1.27e15, "B": 1.27e15, "TN": 1.35e15}
_TR_BW, _TR_LAT = 4.5e12, 8e-6


def _tr_cost(t: torch.Tensor) -> float:
    return t.numel() * t.element_size() * 2 / _TR_BW + _TR_LAT


def _plan(a: torch.Tensor, b: torch.Tensor) -> str:
    """Operand layout for out = a @ b with a = dy^T (a view, K strided) and b = x (K strided)."""
    flops = 2.0 * a.shape[0] * a.shape[1] * b.shape[1]
    cost = {"NN": flops / _PF["NN"],
            "A": flops / _PF["A"] + _tr_cost(a),
            "B": flops / _PF["B"] + _tr_cost(b),
            "TN": flops / _PF["TN"] + _tr_cost(a) + _tr_cost(b)}
    return min(cost, key=cost.get)


def _plannable(a: torch.Tensor, b: torch.Tensor) -> bool:
    return (a.is_cuda and a.dtype in (torch.bfloat16, torch.float16) and a.dim() == 2 and a.stride(0) == 1
            and a.stride(1) != 1
            and b.stride(-1) == 1 and a.shape[0] % 8 == 0 and a.shape[1] % 8 == 0 and b.shape[1] % 8 == 0)


def apply_plan(a: torch.Tensor, b: torch.Tensor, plan: str):
    """Make the operands the plan names K-contiguous (HIP transpose)."""
    if plan in ("A", "TN"):
        a = transpose(a.t())  # [N, T] contiguous
    if plan in ("B", "TN"):
        b = transpose(b).t()  # [T, K] view of a contiguous [K, T]
    return a, b


def grad_mm(out: torch.Tensor, a: torch.Tensor, b: torch.Tensor, acc: bool) -> torch.Tensor:
    """out (+)= a @ b. `out` may be bf16 (scratch, acc must be False) or fp32 (direct accumulation).

    For the weight-gradient shape (a = dy.t() with dy [T, N] row-major, b = x [T, K] row-major) the
    operands whose transpose pays for itself are first made K-contiguous with the HIP transpose.
    fp32 outputs on the GPU then go through hipBLASLt directly with a per-shape tuned solution
    (:func:`lt_mm`).
    """
    if out.is_cuda and _plannable(a, b):
        a, b = apply_plan(a, b, _plan(a, b))
    if out.is_cuda and lt_enabled():
        if a.dtype == torch.bfloat16 and lt_mm(out, a, b, acc):  # tuned per-problem solution (bf16 table)
            return out
        if a.dtype == torch.float16 and out.dtype == torch.float32:
            # fp16 -> fp32 accumulate straight through hipBLASLt with a solution timed on first use: the
            # library's first heuristic pick for these problems is a 32x32 macro-tile kernel that ran
            # ~10 ms per dW GEMM on MI355X (profiles/rocprof_kernel_stats_fp16_heuristic_r02.csv)
            beta = 1.0 if acc else 0.0
            hip_ops().gemm_lt(out, a, b, beta, _f16_solution(out, a, b, beta))
            return out
    if out.dtype == a.dtype:
        if acc:
            return torch.addmm(out, a, b, beta=1.0, out=out)
        return torch.mm(a, b, out=out)
    if out.is_cuda:
        if acc:
            return torch.addmm(out, a, b, beta=1.0, out_dtype=out.dtype, out=out)
        return torch.mm(a, b, out_dtype=out.dtype, out=out)
    r = a.float() @ b.float()
    if acc:
        return out.add_(r)
    return out.copy_(r)


# ---------------------------------------------------------------------------------------------
# hipBLASLt with per-shape solution choice (csrc/kernels/gemm_lt.hip) for the fp32-output dW GEMMs
_LT: dict = {"table": None, "version": None, "timings": {}}


def lt_enabled() -> bool:
    """hipBLASLt through csrc/kernels/gemm_lt.hip whenever the native library is loaded."""
    return hip_available()


def _lt_key(out: torch.Tensor, a: torch.Tensor, b: torch.Tensor, beta: float) -> str:
    def lay(t):
        return f"N{t.stride(0)}" if t.stride(1) == 1 else f"T{t.stride(1)}"
    return (f"{a.shape[0]}x{b.shape[1]}x{a.shape[1]}:{lay(a)}:{lay(b)}:{str(out.dtype)[6:]}{out.stride(0)}"
            f":beta{int(beta != 0)}")


def _lt_table() -> dict:
    """Tuned solution indices for this hipBLASLt build (tools/tune_gemm_lt.py), keyed by problem."""
    if _LT["table"] is None:
        ver = int(hip_ops().gemm_lt_version())
        _LT["version"] = ver
        _LT["table"] = {}
        path = TUNED_DIR / f"gemm_lt_v{ver}.json"
        if path.exists():
            with open(path) as f:
                _LT["table"].update(json.load(f).get("solutions", {}))
    return _LT["table"]


def lt_mm(out: torch.Tensor, a: torch.Tensor, b: torch.Tensor, acc: bool) -> bool:
    """out (+)= a @ b through hipBLASLt with the solution tuned for this exact problem, if the table
    (tools/bench_gemm_lt.py --write) has one; False = not tuned, the caller takes the aten path."""
    beta = 1.0 if acc else 0.0
    idx = _lt_table().get(_lt_key(out, a, b, beta))
    if idx is None or idx < 0:
        return False
    hip_ops().gemm_lt(out, a, b, beta, idx)
    return True


_F16_PICK: dict = {}


def _f16_cache_path() -> Path:
    base = os.environ.get("DLGM_TUNE_CACHE") or os.path.join(os.path.expanduser("~"), ".cache", "dlgm")
    _lt_table()
    return Path(base) / f"gemm_lt_f16_v{_LT['version']}.json"


def _f16_load() -> None:
    """Recorded fp16 picks: the committed table (tuned/gemm_lt_f16_v<ver>.json) first, then this host's cache."""
    if _F16_PICK:
        return
    _lt_table()
    for path in (TUNED_DIR / f"gemm_lt_f16_v{_LT['version']}.json", _f16_cache_path()):
        try:
            with open(path) as f:
                for k, v in json.load(f).get("solutions", {}).items():
                    _F16_PICK.setdefault(k, int(v))
        except (OSError, ValueError):
            pass
    _F16_PICK.setdefault("", -1)  # loaded marker


def _f16_persist(key: str, idx: int) -> None:
    """Merge one timed pick into the host cache (atomic replace): every later process reuses it. The
    read-merge-replace holds an exclusive lock on a sidecar file, so ranks tuning at the same time never drop each
    other's picks (a lost pick would be re-timed later and could differ: different bits across processes)."""
    import fcntl
    path = _f16_cache_path()
    try:
        path.parent.mkdir(parents=True, exist_ok=True)
        with open(path.with_suffix(".lock"), "a") as lk:
            fcntl.flock(lk, fcntl.LOCK_EX)
            cur = {}
            if path.exists():
                with open(path) as f:
                    cur = json.load(f).get("solutions", {})
            cur.setdefault(key, idx)
            _F16_PICK[key] = int(cur[key])  # a pick another process recorded first wins here too
            tmp = path.with_suffix(f".{os.getpid()}.tmp")
            with open(tmp, "w") as f:
                json.dump({"solutions": cur}, f, indent=1, sort_keys=True)
            os.replace(tmp, path)
    except (OSError, ValueError):
        pass


def _f16_solution(out: torch.Tensor, a: torch.Tensor, b: torch.Tensor, beta: float) -> int:
    """hipBLASLt solution for this fp16 -> fp32 problem. Timing picks the fastest of the heuristic's top
    candidates, but two candidates within timing noise of each other would make the pick -- and with it the
    summation order, i.e. the bits -- differ from process to process. So a pick is taken from the committed
    table or this host's cache when one is recorded; only a problem seen nowhere is timed, and its pick is
    written to the cache at once, so every later process computes the same bits."""
    _f16_load()
    key = _lt_key(out, a, b, beta)
    idx = _F16_PICK.get(key)
    if idx is None:
        res = hip_ops().gemm_lt_tune(out, a, b, beta, 24, False, 2)
        idx = int(res[0, 0]) if res.shape[0] else -1
        _F16_PICK[key] = idx
        _f16_persist(key, idx)
        idx = _F16_PICK[key]
    return idx


def mm(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a @ b for the forward / input-gradient GEMMs: tuned hipBLASLt solution when one is recorded."""
    if a.is_cuda and a.dtype == torch.bfloat16 and lt_enabled():
        out = torch.empty(a.shape[0], b.shape[1], dtype=a.dtype, device=a.device)
        if lt_mm(out, a, b, False):
            return out
    return torch.mm(a, b)


def grad_copy(out: torch.Tensor, src: torch.Tensor, acc: bool) -> None:
    if acc:
        out.add_(src.to(out.dtype))
    else:
        out.copy_(src)


def transpose(x: torch.Tensor, out: Optional[torch.Tensor] = None, rows: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Contiguous x^T for a 2-D bf16 tensor (register-blocked HIP kernel on the GPU). rows (int32 [R'], optional):
    transpose a re-laid row space instead -- column r of the result is x[rows[r]], zeros where rows[r] < 0."""
    if rows is not None:
        if use_native(x):
            return hip_ops().transpose(x, out, rows)
        s = rows.long()
        xr = x.index_select(0, s.clamp(min=0)) * (s >= 0).unsqueeze(1).to(x.dtype)
        y = xr.t().contiguous()
        return out.copy_(y) if out is not None else y
    if use_native(x) and x.dtype in (torch.bfloat16, torch.float16) and x.shape[0] % 8 == 0 and x.shape[1] % 8 == 0 \
            and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0:
        return hip_ops().transpose(x, out)
    y = x.t().contiguous()
    if out is not None:
        out.copy_(y)
        return out
    return y


def transpose_multi(xs: list, rows: torch.Tensor) -> torch.Tensor:
    """out[C, P]: column p = xs[rows[p] >> 24][rows[p] & 0xFFFFFF] (zeros where rows[p] < 0); xs row-major [R_s, C]
    of one dtype / row stride, at most 8 (csrc/kernels/transpose.hip, one launch)."""
    if use_native(xs[0]):
        return hip_ops().transpose_multi(list(xs), rows)
    r = rows.long()
    valid = r >= 0
    s, i = (r >> 24).clamp(min=0), (r & 0xFFFFFF)
    C = xs[0].shape[1]
    out = torch.zeros(C, r.numel(), dtype=xs[0].dtype)
    for t, x in enumerate(xs):
        m = valid & (s == t)
        out[:, m] = x[i[m]].t()
    return out


def dx_mm(dy: torch.Tensor, p: dict, name: str) -> torch.Tensor:
    """Input gradient dy @ W for a weight stored [out, in]. When the engine supplies the cached
    transpose ``p[name + ".T"]`` ([in, out], refreshed once per optimizer step) the GEMM runs as
    dy @ (W^T)^T -- both operands K-contiguous, hipBLASLt's fastest layout on gfx950."""
    wt = p.get(name + ".T")
    if wt is not None:
        return mm(dy, wt.t())
    return mm(dy, p[name])
