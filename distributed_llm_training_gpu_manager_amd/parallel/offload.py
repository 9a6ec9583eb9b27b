"""ZeRO-Offload: the fp32 optimizer partition in host memory, updated by the C++ AdamW.

Parity path for the reference's ``offload_optimizer`` knob
(``ai_engine/deepspeed_launcher.py:197-212``; default ``OffloadDevice.CPU`` at ``:39``;
presets 7b/13b/70b at ``:372-407``) -- SURVEY.md §2.5 N2/N3, §2.7 C9. On MI355X the
288 GB of HBM3E holds the full Llama-3-70B optimizer partition at W = 8, so this is
not the hot path; it exists so that every reference config runs.

Layout
    master, exp_avg, exp_avg_sq  fp32 [shard_total]   pinned host RAM ("cpu"), or
                                                        file-backed mmap under nvme_path ("nvme")
    grad_shard, p16_shard         stay on the GPU

Step (one HIP side stream, two pinned staging slots per direction)
    D2H  grad chunk i+1      (copy engine)
    CPU  AdamW chunk i       (csrc/host/ckpt_io.cpp dlgm_cpu_adamw: AVX2/FMA, OpenMP)
    H2D  bf16 params chunk i-1
so PCIe traffic in both directions overlaps the host update.

NVMe ("nvme"): the three state files are swapped through ``buffer_count`` (reference default 4,
``deepspeed_launcher.py:201``) host staging slots by the C++ AIO engine (csrc/host/aio.cpp, the
DeepSpeed ``aio`` op's role): reads of chunk i+buffer_count-2 and the write-back of chunk i-1 are
in flight while chunk i is updated, so host RAM holds only the ring, not the optimizer state. The
files are also mapped (``master`` / ``exp_avg`` / ``exp_avg_sq`` tensors) for the cold paths --
initialisation, checkpoint capture / restore, consolidation -- which share the page cache with
the engine's buffered I/O and therefore always see the swapped state.
"""
from __future__ import annotations

import os
import time
from typing import Dict, List, Optional, Tuple

import torch

from .. import _host
from ..utils.streams import owned_stream

CHUNK_ELEMS = 32 << 20  # 128 MiB of fp32 gradient per staging slot


class HostOffloadOptimizer:
    def __init__(self, numel: int, device: torch.device, kind: str = "cpu", nvme_path: Optional[str] = None,
                 rank: int = 0, chunk_elems: int = CHUNK_ELEMS, buffer_count: int = 4, aio_threads: int = 8,
                 aio_block_size: int = 8 << 20, dtype: torch.dtype = torch.bfloat16):
        assert kind in ("cpu", "nvme"), kind
        self.dtype = dtype  # the compute copy: bf16 (AdamW writes it in the host update) or fp16
        if _host.lib() is None:
            raise RuntimeError("optimizer offload needs the host runtime (_dlgm_host.so); run build()")
        self.n, self.device, self.kind = numel, device, kind
        self.cuda = device.type == "cuda"
        self.chunk = max(1, min(chunk_elems, numel))
        self.files: List[str] = []
        self.aio: Optional[_host.Aio] = None
        if kind == "nvme":
            root = nvme_path or os.environ.get("DLGM_NVME_PATH", "/tmp/dlgm_nvme")
            os.makedirs(root, exist_ok=True)
            self.master, self.exp_avg, self.exp_avg_sq = (self._mmap(root, rank, nm) for nm in
                                                          ("master", "exp_avg", "exp_avg_sq"))
            self.aio = _host.Aio(aio_threads, aio_block_size)
            self.fh = [self.aio.open(p, self.n * 4) for p in self.files]
            self.nbuf = max(3, int(buffer_count))
            self.sslot = [_host.aligned_empty(3 * self.chunk).view(3, self.chunk) for _ in range(self.nbuf)]
            self.swap_stats = {"read_GiB": 0.0, "write_GiB": 0.0, "io_wait_s": 0.0}
        else:
            mk = lambda: torch.zeros(numel, dtype=torch.float32, pin_memory=self.cuda)  # noqa: E731
            self.master, self.exp_avg, self.exp_avg_sq = mk(), mk(), mk()
        if self.cuda:
            self.stream = owned_stream(device, "offload", owner=self)
            self.gslot = [torch.empty(self.chunk, dtype=torch.float32, pin_memory=True) for _ in range(2)]
            self.pslot = [torch.empty(self.chunk, dtype=dtype, pin_memory=True) for _ in range(2)]

    def _mmap(self, root: str, rank: int, name: str) -> torch.Tensor:
        path = os.path.join(root, f"zero_offload_r{rank}.{name}.f32")
        with open(path, "wb") as f:
            f.truncate(self.n * 4)  # sparse file: zeros
        self.files.append(path)
        return torch.from_file(path, shared=True, size=self.n, dtype=torch.float32)

    def host_bytes(self) -> int:
        return 3 * self.n * 4

    # ------------------------------------------------------------------ params
    def push_params(self, p16_shard: torch.Tensor) -> None:
        """p16_shard <- bf16(master) (initialisation / restore)."""
        for off in range(0, self.n, self.chunk):
            ln = min(self.chunk, self.n - off)
            p16_shard.narrow(0, off, ln).copy_(self.master.narrow(0, off, ln).to(p16_shard.dtype))

    # ------------------------------------------------------------------ step
    def step(self, grad_shard: torch.Tensor, p16_shard: torch.Tensor, *, lr: float, beta1: float, beta2: float,
             eps: float, weight_decay: float, step: int, gscale: float) -> None:
        bc1 = 1.0 - beta1 ** step
        bc2 = 1.0 - beta2 ** step
        hyper = (lr, beta1, beta2, eps, weight_decay, bc1, bc2, gscale)
        if not self.cuda and self.kind != "nvme":
            _host.cpu_adamw_(self.master, self.exp_avg, self.exp_avg_sq, grad_shard,
                             p16_shard if p16_shard.dtype == torch.bfloat16 else None, *hyper)
            if p16_shard.dtype != torch.bfloat16:
                p16_shard.copy_(self.master)
            return
        if self.kind == "nvme":
            return self._step_swapped(grad_shard, p16_shard, hyper)
        chunks = [(off, min(self.chunk, self.n - off)) for off in range(0, self.n, self.chunk)]
        cur = torch.cuda.current_stream(self.device)
        s = self.stream
        s.wait_stream(cur)  # gradients final
        d2h: List[Optional[torch.cuda.Event]] = [None] * len(chunks)
        h2d: List[Optional[torch.cuda.Event]] = [None, None]

        def issue_d2h(i: int) -> None:
            off, ln = chunks[i]
            with torch.cuda.stream(s):
                self.gslot[i % 2][:ln].copy_(grad_shard.narrow(0, off, ln), non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(s)
            d2h[i] = ev

        issue_d2h(0)
        for i, (off, ln) in enumerate(chunks):
            if i + 1 < len(chunks):
                issue_d2h(i + 1)  # slot (i+1)%2 was consumed by the host update of chunk i-1
            d2h[i].synchronize()
            slot = i % 2
            if h2d[slot] is not None:
                h2d[slot].synchronize()  # the H2D of chunk i-2 has drained this bf16 staging slot
            self._host_update(self.master.narrow(0, off, ln), self.exp_avg.narrow(0, off, ln),
                              self.exp_avg_sq.narrow(0, off, ln), self.gslot[slot][:ln], self.pslot[slot][:ln], hyper)
            with torch.cuda.stream(s):
                p16_shard.narrow(0, off, ln).copy_(self.pslot[slot][:ln], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(s)
            h2d[slot] = ev
        cur.wait_stream(s)  # compute resumes on the updated bf16 params

    @staticmethod
    def _host_update(master, m, v, g, p16, hyper) -> None:
        """AVX2 AdamW on one chunk; the runtime writes a bf16 compute copy itself, an fp16 one is cast here."""
        if p16 is None or p16.dtype == torch.bfloat16:
            _host.cpu_adamw_(master, m, v, g, p16, *hyper)
        else:
            _host.cpu_adamw_(master, m, v, g, None, *hyper)
            p16.copy_(master)

    def _step_swapped(self, grad_shard: torch.Tensor, p16_shard: torch.Tensor, hyper) -> None:
        """NVMe: state chunks stream file -> ring slot -> AdamW -> file, reads running buffer_count-2
        chunks ahead and writes draining behind; gradients / bf16 params move as in the host path."""
        chunks = [(off, min(self.chunk, self.n - off)) for off in range(0, self.n, self.chunk)]
        nb, ahead = self.nbuf, self.nbuf - 2
        aio = self.aio
        reads: dict = {}
        writes: dict = {}
        waited = 0.0

        def wait_all(tickets) -> None:
            nonlocal waited
            t0 = time.perf_counter()
            for tk in tickets:
                aio.wait(tk)
            waited += time.perf_counter() - t0

        def issue_read(i: int) -> None:
            if i - nb in writes:  # the slot's previous chunk must be on its way to the file first
                wait_all(writes.pop(i - nb))
            off, ln = chunks[i]
            st = self.sslot[i % nb]
            reads[i] = [aio.read(h, st[k, :ln], off * 4) for k, h in enumerate(self.fh)]

        cuda = self.cuda
        if cuda:
            cur = torch.cuda.current_stream(self.device)
            s = self.stream
            s.wait_stream(cur)  # gradients final
            d2h: List[Optional[torch.cuda.Event]] = [None] * len(chunks)
            h2d: List[Optional[torch.cuda.Event]] = [None, None]

            def issue_d2h(i: int) -> None:
                off, ln = chunks[i]
                with torch.cuda.stream(s):
                    self.gslot[i % 2][:ln].copy_(grad_shard.narrow(0, off, ln), non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(s)
                d2h[i] = ev

            issue_d2h(0)
        for i in range(min(ahead, len(chunks))):
            issue_read(i)
        for i, (off, ln) in enumerate(chunks):
            if i + ahead < len(chunks):
                issue_read(i + ahead)
            if cuda and i + 1 < len(chunks):
                issue_d2h(i + 1)
            wait_all(reads.pop(i))
            st = self.sslot[i % nb]
            if cuda:
                d2h[i].synchronize()
                slot = i % 2
                if h2d[slot] is not None:
                    h2d[slot].synchronize()
                g, p16 = self.gslot[slot][:ln], self.pslot[slot][:ln]
            else:
                g = grad_shard.narrow(0, off, ln)
                p16 = p16_shard.narrow(0, off, ln) if p16_shard.dtype == torch.bfloat16 else None
            self._host_update(st[0, :ln], st[1, :ln], st[2, :ln], g, p16, hyper)
            writes[i] = [aio.write(h, st[k, :ln], off * 4) for k, h in enumerate(self.fh)]
            if cuda:
                with torch.cuda.stream(s):
                    p16_shard.narrow(0, off, ln).copy_(p16, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(s)
                h2d[slot] = ev
            elif p16 is None:
                p16_shard.narrow(0, off, ln).copy_(st[0, :ln])
        for i in sorted(writes):
            wait_all(writes.pop(i))  # the mapped views (checkpoint capture) read the page cache from here on
        if cuda:
            cur.wait_stream(s)
        nbytes = self.n * 4 * 3 / 2 ** 30
        self.swap_stats["read_GiB"] += nbytes
        self.swap_stats["write_GiB"] += nbytes
        self.swap_stats["io_wait_s"] += waited

    def close(self) -> None:
        if self.aio is not None:
            for h in self.fh:
                self.aio.close(h)
            self.aio.shutdown()
            self.aio = None
        for p in self.files:
            try:
                os.remove(p)
            except OSError:
                pass


class NvmeParamStore:
    """``offload_param.device = "nvme"`` (ZeRO-Infinity parameter offload, reference
    ``ai_engine/deepspeed_launcher.py:205-212``): the rank's 16-bit parameter partition lives in a file under
    ``nvme_path``, not in host RAM.

    Hot paths go through the C++ AIO engine and a ring of ``buffer_count`` pinned slots, each one parameter
    group's shard long:

    * gather: the group's shard is read file -> slot (buffered I/O), then the engine copies it H2D on its
      side stream and all-gathers; a slot is reused only after the H2D that read it has completed (event);
    * read-ahead: the order of the gathers repeats every step (the residency plan is static), so each read
      also issues the AIO read of the shard that followed it last time into the next free slot; the gather
      of that shard then only waits for I/O that has been running meanwhile (DeepSpeed's offload_param
      prefetches partitions ahead of use the same way). A step's writes invalidate read-aheads in flight;
    * after each optimizer step: the new 16-bit values are produced slot by slot (device cast + D2H, or the
      host AdamW's output) and written back with the writes of ``buffer_count - 1`` slots in flight.

    The file is also mapped (``mapped``) for the cold paths -- checkpoint capture / restore, the host
    optimizer's in-place update, tests -- which share the page cache with the buffered AIO descriptor and
    therefore always see the same bytes.
    """

    def __init__(self, numel: int, dtype: torch.dtype, root: Optional[str], rank: int, slot_elems: int,
                 buffer_count: int = 5, cuda: bool = False, aio_threads: int = 8, aio_block_size: int = 8 << 20):
        if _host.lib() is None:
            raise RuntimeError("offload_param=nvme needs the host runtime (_dlgm_host.so); run build()")
        root = root or os.environ.get("DLGM_NVME_PATH", "/tmp/dlgm_nvme")
        os.makedirs(root, exist_ok=True)
        self.n, self.dtype, self.cuda = numel, dtype, cuda
        self.esize = torch.empty((), dtype=dtype).element_size()
        self.path = os.path.join(root, f"zero_param_r{rank}.{str(dtype).split('.')[-1]}")
        with open(self.path, "wb") as f:
            f.truncate(numel * self.esize)
        self.mapped = torch.from_file(self.path, shared=True, size=numel, dtype=dtype)
        self.aio = _host.Aio(aio_threads, aio_block_size)
        self.fh = self.aio.open(self.path, numel * self.esize)
        self.slot_elems = max(1, min(slot_elems, numel))
        nb = max(2, int(buffer_count))
        self.slots = [torch.empty(self.slot_elems, dtype=dtype, pin_memory=cuda) for _ in range(nb)]
        self._used: List[Optional["torch.cuda.Event"]] = [None] * nb  # last H2D out of the slot
        self._writes: List[Optional[int]] = [None] * nb                # AIO write ticket out of the slot
        self._next = 0
        self._ahead: Dict[Tuple[int, int], Tuple[int, int]] = {}  # (off, n) -> (slot, AIO read ticket)
        self._slot_key: List[Optional[Tuple[int, int]]] = [None] * nb  # read-ahead a slot holds
        self._follow: Dict[Tuple[int, int], Tuple[int, int]] = {}  # access -> the access after it last time
        self._prev: Optional[Tuple[int, int]] = None
        self.read_ahead = nb > 2  # one slot in use, one being filled, one for the H2D still draining
        self.stats = {"read_GiB": 0.0, "write_GiB": 0.0, "io_wait_s": 0.0, "read_ahead_hits": 0, "reads": 0}

    def _wait(self, ticket: int) -> None:
        t0 = time.perf_counter()
        self.aio.wait(ticket)
        self.stats["io_wait_s"] += time.perf_counter() - t0

    def _take(self) -> int:
        i = self._next
        self._next = (i + 1) % len(self.slots)
        if self._used[i] is not None:
            self._used[i].synchronize()
            self._used[i] = None
        if self._writes[i] is not None:
            self._wait(self._writes[i])
            self._writes[i] = None
        key = self._slot_key[i]
        if key is not None:  # an unused read-ahead in this slot: let it finish, then forget it
            self._wait(self._ahead.pop(key)[1])
            self._slot_key[i] = None
        return i

    def read(self, off: int, n: int):
        """Read elements [off, off + n) into a slot (or take the read-ahead of it); returns (slot, host view)."""
        assert n <= self.slot_elems, (n, self.slot_elems)
        key = (off, n)
        self.stats["reads"] += 1
        if key in self._ahead:
            i, tk = self._ahead.pop(key)
            self._slot_key[i] = None
            self._wait(tk)
            self.stats["read_ahead_hits"] += 1
        else:
            i = self._take()
            self._wait(self.aio.read(self.fh, self.slots[i][:n], off * self.esize))
            self.stats["read_GiB"] += n * self.esize / 2 ** 30
        t = self.slots[i][:n]
        if self._prev is not None:
            self._follow[self._prev] = key
        self._prev = key
        nxt = self._follow.get(key)
        if self.read_ahead and nxt is not None and nxt not in self._ahead and nxt != key:
            j = self._take()
            if j == i:  # never refill the slot just handed out (only possible with a 1-slot ring)
                return i, t
            self._ahead[nxt] = (j, self.aio.read(self.fh, self.slots[j][:nxt[1]], nxt[0] * self.esize))
            self._slot_key[j] = nxt
            self.stats["read_GiB"] += nxt[1] * self.esize / 2 ** 30
        return i, t

    def release_after(self, i: int, ev) -> None:
        """The slot may be refilled once `ev` (the H2D copy out of it) has completed."""
        self._used[i] = ev

    def drop_read_ahead(self) -> None:
        """Forget the read-aheads in flight (the partition is about to change under them)."""
        for key, (i, tk) in list(self._ahead.items()):
            self._wait(tk)
            self._slot_key[i] = None
        self._ahead.clear()
        self._prev = None

    def write(self, produce) -> None:
        """Stream the whole partition back: produce(off, ln, slot_view) fills each slot-sized piece."""
        self.drop_read_ahead()
        for off in range(0, self.n, self.slot_elems):
            ln = min(self.slot_elems, self.n - off)
            i = self._take()
            t = self.slots[i][:ln]
            produce(off, ln, t)
            self._writes[i] = self.aio.write(self.fh, t, off * self.esize)
            self.stats["write_GiB"] += ln * self.esize / 2 ** 30
        self.flush()

    def flush(self) -> None:
        for i, tk in enumerate(self._writes):
            if tk is not None:
                self._wait(tk)
                self._writes[i] = None

    def close(self) -> None:
        if self.aio is not None:
            self.flush()
            self.aio.close(self.fh)
            self.aio.shutdown()
            self.aio = None


class ActivationOffloader:
    """``cpu_checkpointing`` (reference ``activation_checkpointing.cpu_checkpointing``, 70b preset,
    ``deepspeed_launcher.py:215-223, :403``): the per-unit checkpointed inputs kept for recompute
    are streamed to pinned host memory on a side HIP stream during the forward and streamed back,
    one unit ahead, during the backward."""

    def __init__(self, device: torch.device):
        self.device = device
        self.cuda = device.type == "cuda"
        self.stream = owned_stream(device, "offload", owner=self) if self.cuda else None
        self._pool: dict = {}

    def _host_buf(self, t: torch.Tensor) -> torch.Tensor:
        key = (tuple(t.shape), t.dtype)
        free = self._pool.setdefault(key, [])
        return free.pop() if free else torch.empty(t.shape, dtype=t.dtype, pin_memory=self.cuda)

    def _map(self, x, fn):
        if x is None:
            return None
        if isinstance(x, torch.Tensor):
            return fn(x)
        return tuple(self._map(e, fn) for e in x)

    def push(self, x):
        """Start the D2H copy of `x` (tensor / tuple of tensors / None); returns a handle."""
        if not self.cuda:
            return ("host", self._map(x, lambda t: self._host_buf(t).copy_(t)), None, None)
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            host = self._map(x, lambda t: self._host_buf(t).copy_(t, non_blocking=True))
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return ("host", host, ev, x)  # keep the device tensors alive until the copy has drained

    def release_device(self, h):
        """Drop the device copy once its D2H has finished (call after the next unit's forward)."""
        if h[0] != "host" or h[3] is None:
            return h
        h[2].synchronize()
        return ("host", h[1], None, None)

    def prefetch(self, h):
        """Start the H2D copy back; returns a handle for :meth:`get`."""
        if h[0] != "host":
            return h
        host = h[1]
        if not self.cuda:
            return ("dev", host, None, host)
        if h[2] is not None:
            self.stream.wait_event(h[2])
        with torch.cuda.stream(self.stream):
            dev = self._map(host, lambda t: t.to(self.device, non_blocking=True))
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return ("dev", dev, ev, host)

    def get(self, h):
        if h[0] == "host":
            h = self.prefetch(h)
        _, dev, ev, host = h
        if ev is not None:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(ev)
            self._map(dev, lambda t: t.record_stream(cur))  # allocated on the side stream, consumed here
            ev.synchronize()  # the host staging buffers may be reused after this
        self._map(host, lambda t: self._pool.setdefault((tuple(t.shape), t.dtype), []).append(t))
        return dev
