"""Stream-ordering audit: a vector-clock race detector for HIP streams (``DLGM_STREAM_AUDIT=1``).

SURVEY.md §5.2 asks for "stream-ordering asserts in debug mode". The engine overlaps work on several HIP streams
(communicators, the W^T-cache and MoE re-layout side streams, the overlapped optimizer, the checkpoint copy stream) and
orders them with events, ``wait_stream`` and ``record_stream``. A missing edge does not fail deterministically: it
fails when the GPU happens to schedule the two queues against each other. This module checks
the edges themselves, independent of timing, the way ThreadSanitizer checks threads:

* every stream S carries a vector clock ``vc[S]``; each op enqueued on S advances ``vc[S][S]``;
* ``Event.record(S)`` snapshots ``vc[S]``; ``Event.wait(T)`` / ``T.wait_stream(S)`` join the snapshot into ``vc[T]``;
* a host synchronisation (``torch.cuda.synchronize``, ``Stream/Event.synchronize``, a completed ``Event.query``, a
  blocking device-to-host copy, ``.item()``) joins into a host clock that every later op inherits;
* each access to device memory is recorded per storage and byte range with the stream and tick that made it. An access
  on stream T conflicts with an earlier access on stream S to overlapping bytes (at least one a write) unless
  ``vc[T][S]`` has reached that tick: a read-after-write, write-after-read or write-after-write **race**. Page-locked
  host memory is tracked as well: H2D / D2H copies access it on their stream, CPU ops on it run on a ``host`` key
  that is complete when the op returns (a CPU write into a buffer an earlier async D2H / H2D still uses is a race);
* the caching allocator hands a freed block back to the stream that allocated it without waiting for other streams,
  unless the tensor was ``record_stream``-ed to them. When a new storage occupies bytes of a dead one, the dead
  storage's accesses on other streams (not covered by ``record_stream``) must be ordered before every access to the
  new storage: otherwise it is a **use-after-free** race -- the buffer is rewritten while another queue still reads
  (or writes) the old tensor.

Reads and writes come from the op schemas (``Tensor(a!)`` arguments and outputs are writes), so the native ``dlgm::``
ops are covered as well as aten. Not modelled: RCCL / c10d collectives (they run on ProcessGroupNCCL's streams and are
ordered by ``work.wait()``), memory touched through ctypes (the checkpoint DMA), and work captured into HIP graphs
(the audit pauses during capture). Missing host synchronisations only make the audit stricter (more reports, never
fewer).

Usage::

    with stream_audit() as audit:
        ...                              # any GPU code
    assert not audit.hazards, audit.report()

``tests/conftest.py`` wraps every GPU test in it when ``DLGM_STREAM_AUDIT=1``. The clock model itself
(:class:`HazardModel`) is plain Python with opaque stream keys, tested on the CPU (``tests/test_stream_audit.py``).
"""
from __future__ import annotations

import bisect
import contextlib
import os
import traceback
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, Hashable, List, Optional, Tuple

Clock = Dict[Hashable, int]

# access records kept per storage (oldest dropped first: a bounded detector, never a false report); raise it with
# DLGM_STREAM_AUDIT_RECORDS for a deeper (slower) pass over buffers touched through many views
MAX_RECORDS = int(os.environ.get("DLGM_STREAM_AUDIT_RECORDS", "48"))


def enabled() -> bool:
    return os.environ.get("DLGM_STREAM_AUDIT", "0") == "1"


def _join(a: Clock, b: Clock) -> None:
    for k, v in b.items():
        if a.get(k, 0) < v:
            a[k] = v


@dataclass
class Access:
    lo: int
    hi: int
    stream: Hashable
    tick: int
    write: bool
    what: str


@dataclass
class Hazard:
    kind: str  # "RAW" | "WAR" | "WAW" | "reuse"
    storage: str
    first: str  # the earlier access: op, stream, tick
    second: str  # the later, unordered access
    where: str = ""

    def __str__(self) -> str:
        return f"{self.kind} on {self.storage}: {self.second} is not ordered after {self.first}" + \
            (f"\n{self.where}" if self.where else "")


@dataclass
class StorageRec:
    name: str
    base: int
    nbytes: int
    alloc_stream: Hashable
    alive: Callable[[], bool]
    accesses: List[Access] = field(default_factory=list)
    last_by_stream: Clock = field(default_factory=dict)  # stream -> newest tick of any access
    record_streams: set = field(default_factory=set)
    # (stream, tick, what) of a dead storage's accesses that every access to this one must follow
    pending: List[Tuple[Hashable, int, str]] = field(default_factory=list)


class HazardModel:
    """Vector clocks over opaque stream keys, per-storage access histories, allocator-reuse checks."""

    def __init__(self, max_hazards: int = 64, stack: bool = False):
        self.vc: Dict[Hashable, Clock] = {}
        self.host: Clock = {}
        self.recs: Dict[Hashable, StorageRec] = {}
        self._starts: List[int] = []  # sorted bases of tracked storages (live or dead), for reuse detection
        self._by_start: Dict[int, List[Hashable]] = {}
        self._max_span = 0
        self.hazards: List[Hazard] = []
        self.max_hazards = max_hazards
        self.stack = stack
        self.ops = 0

    # ---------------------------------------------------------------- clocks
    def _clock(self, s: Hashable) -> Clock:
        c = self.vc.get(s)
        if c is None:
            c = self.vc[s] = {}
        return c

    def enqueue(self, s: Hashable) -> int:
        """One op queued on stream s: it follows everything the host has seen complete. Returns its tick."""
        c = self._clock(s)
        _join(c, self.host)
        c[s] = c.get(s, 0) + 1
        self.ops += 1
        return c[s]

    def snapshot(self, s: Hashable) -> Clock:
        """Event.record on s."""
        return dict(self._clock(s))

    def wait(self, s: Hashable, snap: Optional[Clock]) -> None:
        """Stream s waits for an event snapshot (Event.wait / Stream.wait_event / wait_stream)."""
        if snap:
            _join(self._clock(s), snap)

    def host_sync(self, snap: Optional[Clock]) -> None:
        """The host observed a snapshot complete (stream / event / device synchronize, blocking D2H copy)."""
        if snap:
            _join(self.host, snap)

    def device_sync(self) -> None:
        for c in self.vc.values():
            _join(self.host, c)

    def _ordered(self, s: Hashable, other: Hashable, tick: int) -> bool:
        return other == s or self._clock(s).get(other, 0) >= tick or self.host.get(other, 0) >= tick

    # ---------------------------------------------------------------- storages
    def storage(self, key: Hashable, base: int, nbytes: int, stream: Hashable, alive: Callable[[], bool],
                name: str = "", reuse: bool = True) -> StorageRec:
        """The record of a storage, created (with the reuse check armed unless `reuse` is False: pinned host blocks,
        which the host caching allocator hands out again only after the streams that copied them are done) the first
        time it is seen."""
        rec = self.recs.get(key)
        if rec is not None and rec.alive() and rec.base == base:
            return rec
        cands = []
        if rec is not None:  # a dead storage whose key was recycled: still a candidate for the reuse check
            self._forget(key, rec)
            cands.append((None, rec))
        cands += [(k, self.recs[k]) for k in self._overlapping(base, base + nbytes)]
        new = StorageRec(name or f"storage@{base:#x}+{nbytes}", base, nbytes, stream, alive)
        for k, old in cands:
            if old.alive() or old.base >= base + nbytes or old.base + old.nbytes <= base:
                continue
            for s, t in (old.last_by_stream.items() if reuse else ()):
                if s in old.record_streams:
                    continue  # the allocator itself waited for these before handing the block out again
                new.pending.append((s, t, old.name))
            if k is not None:
                self._forget(k, old)
        self.recs[key] = new
        bisect.insort(self._starts, base)
        self._by_start.setdefault(base, []).append(key)
        self._max_span = max(self._max_span, nbytes)
        return new

    def _overlapping(self, lo: int, hi: int) -> List[Hashable]:
        """Keys of tracked storages overlapping [lo, hi): those starting below hi, walked back while one could
        still reach lo (no tracked storage is longer than the longest seen)."""
        out = []
        j = bisect.bisect_left(self._starts, hi) - 1
        prev = None
        while j >= 0:
            b = self._starts[j]
            if b + self._max_span <= lo:
                break
            if b != prev:
                for k in self._by_start.get(b, ()):
                    r = self.recs.get(k)
                    if r is not None and b + r.nbytes > lo:
                        out.append(k)
            prev = b
            j -= 1
        return out

    def _forget(self, key: Hashable, rec: StorageRec) -> None:
        self.recs.pop(key, None)
        keys = self._by_start.get(rec.base)
        if keys and key in keys:
            keys.remove(key)
            if not keys:
                del self._by_start[rec.base]
                i = bisect.bisect_left(self._starts, rec.base)
                if i < len(self._starts) and self._starts[i] == rec.base:
                    self._starts.pop(i)

    def record_stream(self, rec: StorageRec, s: Hashable) -> None:
        rec.record_streams.add(s)

    # ---------------------------------------------------------------- accesses
    def access(self, rec: StorageRec, lo: int, hi: int, s: Hashable, tick: int, write: bool, what: str) -> None:
        mine = f"{'write' if write else 'read'} by {what} (stream {_sname(s)}, tick {tick})"
        if rec.pending:
            keep = []
            for (ps, pt, pname) in rec.pending:
                if self.host.get(ps, 0) >= pt:
                    continue
                if not self._ordered(s, ps, pt):
                    self._report("reuse", rec, f"the last access to freed {pname} on stream {_sname(ps)} (tick {pt})",
                                 mine)
                keep.append((ps, pt, pname))
            rec.pending = keep
        for a in rec.accesses:
            if a.stream == s or a.hi <= lo or a.lo >= hi or not (write or a.write):
                continue
            if not self._ordered(s, a.stream, a.tick):
                kind = "WAW" if (write and a.write) else ("RAW" if a.write else "WAR")
                self._report(kind, rec, f"{'write' if a.write else 'read'} by {a.what} (stream {_sname(a.stream)}, "
                                        f"tick {a.tick})", mine)
        acc = rec.accesses
        # drop what every queue has provably finished and what a newer write of this stream covers
        if len(acc) >= MAX_RECORDS // 2:
            acc[:] = [a for a in acc if self.host.get(a.stream, 0) < a.tick and
                      not (write and a.stream == s and a.lo >= lo and a.hi <= hi)]
            if len(acc) >= MAX_RECORDS:
                del acc[:len(acc) - MAX_RECORDS + 1]
        acc.append(Access(lo, hi, s, tick, write, what))
        if rec.last_by_stream.get(s, 0) < tick:
            rec.last_by_stream[s] = tick

    def _report(self, kind: str, rec: StorageRec, first: str, second: str) -> None:
        if len(self.hazards) >= self.max_hazards:
            return
        where = "".join(traceback.format_stack(limit=14)[:-3]) if self.stack else ""
        self.hazards.append(Hazard(kind, rec.name, first, second, where))

    def report(self) -> str:
        if not self.hazards:
            return f"stream audit: no hazards ({self.ops} ops)"
        return f"stream audit: {len(self.hazards)} hazard(s) in {self.ops} ops\n" + \
            "\n".join(f"  [{i}] {h}" for i, h in enumerate(self.hazards))


HOST = "host"  # the stream key of CPU ops on page-locked host memory
_NAMES: Dict[Hashable, str] = {}  # stream key -> name (utils/streams.py registers every named stream here)
# storage base pointer -> why: memory whose cross-stream accesses are ordered by a device-side protocol (atomics,
# flags polled by the kernels themselves) rather than by stream edges; the audit does not track it
_PROTOCOL: Dict[int, str] = {}


def protocol_memory(t, why: str) -> None:
    """Declare `t`'s storage synchronised by a device-side protocol (e.g. the xGMI mesh's state words)."""
    _PROTOCOL[int(t.untyped_storage().data_ptr())] = why


def _sname(s: Hashable) -> str:
    return _NAMES.get(s, f"{s:#x}" if isinstance(s, int) else str(s))


# ------------------------------------------------------------------------------------------- torch binding
def _make_mode(model: HazardModel, fake_stream: Optional[Callable[[], Hashable]] = None):
    """A TorchDispatchMode that feeds every CUDA op's reads / writes into `model`. ``fake_stream`` (CPU tests of this
    binding): audit CPU tensors instead, on the stream key that callable returns."""
    import torch
    from torch.multiprocessing.reductions import StorageWeakRef
    from torch.utils._python_dispatch import TorchDispatchMode

    aten = torch.ops.aten
    factories = {aten.empty.memory_format, aten.empty_strided.default, aten.empty_like.default,
                 aten.new_empty.default, aten.new_empty_strided.default}
    syncing = {aten._local_scalar_dense.default, aten.nonzero.default, aten.equal.default,
               aten.is_nonzero.default}
    schema_cache: Dict[Any, Tuple[List[bool], List[bool]]] = {}

    def pinned(t: "torch.Tensor") -> bool:
        try:
            return t.device.type == "cpu" and t.is_pinned()
        except Exception:
            return False
    # page-locked host memory is tracked too: copies to / from it are accesses on their stream, CPU ops on it are
    # accesses by the host (HOST), complete when they return (e.g. a D2H into a pinned buffer that the next H2D reads)
    dev_ok = (lambda t: not t.is_cuda) if fake_stream is not None else (lambda t: t.is_cuda or pinned(t))

    def flags(func):
        f = schema_cache.get(func)
        if f is None:
            sch = func._schema
            arg_w = [bool(a.alias_info is not None and a.alias_info.is_write) for a in sch.arguments]
            ret_alias = [r.alias_info is not None for r in sch.returns]
            f = schema_cache[func] = (arg_w, ret_alias)
        return f

    def tensors(x):
        if isinstance(x, torch.Tensor):
            yield x
        elif isinstance(x, (list, tuple)):
            for v in x:
                yield from tensors(v)

    def stream_key(s) -> int:
        if hasattr(s, "cuda_stream"):
            return int(s.cuda_stream)
        cs = torch.cuda.Stream(stream_id=s.stream_id, device_index=s.device_index, device_type=s.device_type)
        return int(cs.cuda_stream)

    def tracked(t: "torch.Tensor") -> bool:
        return dev_ok(t) and int(t.untyped_storage().data_ptr()) not in _PROTOCOL

    def rec_of(t: "torch.Tensor", s: Hashable):
        st = t.untyped_storage()
        ref = StorageWeakRef(st)
        host = fake_stream is None and not t.is_cuda
        return model.storage(ref.cdata, st.data_ptr(), st.nbytes(), s, lambda r=ref: not r.expired(),
                             f"{tuple(t.shape)} {str(t.dtype)[6:]} {'pinned ' if host else ''}storage@{st.data_ptr():#x}",
                             reuse=not host)

    def span(t: "torch.Tensor") -> Tuple[int, int]:
        es = t.element_size()
        lo = t.storage_offset() * es
        if t.numel() == 0:
            return lo, lo
        ext = sum((n - 1) * abs(st) for n, st in zip(t.shape, t.stride())) + 1
        return lo, lo + ext * es

    class Mode(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            kwargs = kwargs or {}
            out = func(*args, **kwargs)
            try:
                self._audit(func, args, kwargs, out)
            except Exception as e:  # the audit must never break the program it watches
                model.hazards.append(Hazard("audit-error", str(func), repr(e), ""))
            return out

        def _audit(self, func, args, kwargs, out):
            if fake_stream is None and (not torch.cuda.is_available() or torch.cuda.is_current_stream_capturing()):
                return
            name = str(func.name()) if hasattr(func, "name") else str(func)
            if name.startswith("c10d::"):
                return
            dev_t = tracked
            cuda_in = [t for t in tensors(list(args) + list(kwargs.values())) if dev_ok(t)]
            outs = [t for t in tensors(out) if isinstance(t, torch.Tensor) and dev_ok(t)]
            if not cuda_in and not outs:
                return
            if fake_stream is not None:
                s: Hashable = fake_stream()
            else:
                gpu = [t for t in cuda_in + outs if t.is_cuda]
                s = int(torch.cuda.current_stream(gpu[0].device).cuda_stream) if gpu else HOST
            if func is aten.record_stream.default:
                model.record_stream(rec_of(args[0], s), stream_key(args[1]))
                return
            tick = model.enqueue(s)
            what = name.split("::")[-1]
            if func in factories:
                for t in outs:
                    rec_of(t, s)  # allocation only: no bytes are touched
                return
            try:
                arg_w, ret_alias = flags(func)
            except Exception:
                arg_w, ret_alias = [], []
            if any(ret_alias) and not any(arg_w):
                return  # a view (slice, narrow, view, t, detach, split, ...): no bytes are touched
            sch_args = func._schema.arguments if hasattr(func, "_schema") else []
            written = set()
            for i, a in enumerate(args):
                w = i < len(arg_w) and arg_w[i]
                for t in tensors(a):
                    if dev_t(t):
                        if w:
                            written.add(id(t))
                        lo, hi = span(t)
                        model.access(rec_of(t, s), lo, hi, s, tick, w, what)
            for k, a in kwargs.items():
                idx = next((j for j, sa in enumerate(sch_args) if sa.name == k), None)
                w = idx is not None and idx < len(arg_w) and arg_w[idx]
                for t in tensors(a):
                    if dev_t(t):
                        if w:
                            written.add(id(t))
                        lo, hi = span(t)
                        model.access(rec_of(t, s), lo, hi, s, tick, w, what)
            for t in outs:  # results (in-place results are the written argument itself)
                if id(t) in written or not tracked(t):
                    continue
                lo, hi = span(t)
                model.access(rec_of(t, s), lo, hi, s, tick, True, what)
            # blocking device -> host traffic: the host has seen this stream's work complete
            host_out = fake_stream is None and (
                any(isinstance(t, torch.Tensor) and not t.is_cuda for t in tensors(out)) or
                any(isinstance(a, torch.Tensor) and not a.is_cuda for a in args[:1]))
            nb = bool(kwargs.get("non_blocking", False)) or (len(args) > 2 and args[2] is True and
                                                            func is aten.copy_.default)
            if s == HOST:  # a CPU op on pinned memory has completed when it returns
                model.host_sync({HOST: tick})
            elif func in syncing or (cuda_in and host_out and not nb and func in (aten._to_copy.default,
                                                                                   aten.copy_.default)):
                model.host_sync(model.snapshot(s))

    return Mode()


_PATCHED: Dict[str, Any] = {}
_ACTIVE: List[HazardModel] = []


def _install_event_hooks() -> None:
    """Route Event.record / wait / synchronize / query and stream / device synchronisation into the active model."""
    import torch

    if _PATCHED:
        return
    Ev, St = torch.cuda.Event, torch.cuda.Stream
    _PATCHED.update(record=Ev.record, wait=Ev.wait, esync=Ev.synchronize, query=Ev.query, ssync=St.synchronize,
                    dsync=torch.cuda.synchronize)

    def cur(stream):
        return stream if stream is not None else torch.cuda.current_stream()

    def record(self, stream=None):
        _PATCHED["record"](self, stream)
        if _ACTIVE and not torch.cuda.is_current_stream_capturing():
            s = int(cur(stream).cuda_stream)
            m = _ACTIVE[-1]
            m.enqueue(s)
            self._dlgm_audit_snap = m.snapshot(s)

    def wait(self, stream=None):
        _PATCHED["wait"](self, stream)
        if _ACTIVE and not torch.cuda.is_current_stream_capturing():
            _ACTIVE[-1].wait(int(cur(stream).cuda_stream), getattr(self, "_dlgm_audit_snap", None))

    def esync(self):
        _PATCHED["esync"](self)
        if _ACTIVE:
            _ACTIVE[-1].host_sync(getattr(self, "_dlgm_audit_snap", None))

    def query(self):
        done = _PATCHED["query"](self)
        if done and _ACTIVE:
            _ACTIVE[-1].host_sync(getattr(self, "_dlgm_audit_snap", None))
        return done

    def ssync(self):
        _PATCHED["ssync"](self)
        if _ACTIVE:
            m = _ACTIVE[-1]
            m.host_sync(m.snapshot(int(self.cuda_stream)))

    def dsync(device=None):
        _PATCHED["dsync"](device)
        if _ACTIVE:
            _ACTIVE[-1].device_sync()

    Ev.record, Ev.wait, Ev.synchronize, Ev.query, St.synchronize = record, wait, esync, query, ssync
    torch.cuda.synchronize = dsync


def _remove_event_hooks() -> None:
    import torch

    if not _PATCHED or _ACTIVE:
        return
    Ev, St = torch.cuda.Event, torch.cuda.Stream
    Ev.record, Ev.wait, Ev.synchronize, Ev.query = _PATCHED["record"], _PATCHED["wait"], _PATCHED["esync"], \
        _PATCHED["query"]
    St.synchronize = _PATCHED["ssync"]
    torch.cuda.synchronize = _PATCHED["dsync"]
    _PATCHED.clear()


@contextlib.contextmanager
def stream_audit(stack: bool = False, name_streams: bool = True):
    """Audit every CUDA op issued inside the block; the model's ``hazards`` list is filled in place."""
    import torch

    model = HazardModel(stack=stack)
    if not torch.cuda.is_available():
        yield model
        return
    if name_streams:
        _NAMES[int(torch.cuda.current_stream().cuda_stream)] = "compute"
    _install_event_hooks()
    _ACTIVE.append(model)
    mode = _make_mode(model)
    try:
        with mode:
            yield model
    finally:
        _ACTIVE.remove(model)
        _remove_event_hooks()


# ------------------------------------------------------------------------------------------- poisoned allocations
def poison_enabled() -> bool:
    return os.environ.get("DLGM_POISON_ALLOC", "0") == "1"


@contextlib.contextmanager
def poison_allocations(value: float = float("nan")):
    """Every floating-point tensor created by an uninitialised factory op (``empty``, ``empty_like``, ``new_empty``,
    ``empty_strided``) inside the block is filled with NaN on the allocating stream before anyone can read it
    (``DLGM_POISON_ALLOC=1`` in tests/conftest.py). The caching allocator hands out recycled blocks whose old bytes
    depend on what the process ran before; code that reads such bytes (a GEMM accumulating with beta = 1 into a fresh
    buffer, a missing zero-fill, a partly written output) then computes different numbers after a different process
    history -- the signature of the round-4 "first engine differs" mismatch. With the poison the same read turns into
    NaN every time. Integer and bool tensors are left alone (poisoned indices would fault the GPU)."""
    import torch
    from torch.utils._python_dispatch import TorchDispatchMode

    if not torch.cuda.is_available():
        yield
        return
    aten = torch.ops.aten
    factories = {aten.empty.memory_format, aten.empty_strided.default, aten.empty_like.default,
                 aten.new_empty.default, aten.new_empty_strided.default}

    class Poison(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            out = func(*args, **(kwargs or {}))
            if func in factories and isinstance(out, torch.Tensor) and out.is_floating_point() and out.numel() > 0 \
                    and (out.is_cuda or (out.device.type == "cpu" and out.is_pinned())):  # pinned staging too
                out.fill_(value)
            return out

    with Poison():
        yield
