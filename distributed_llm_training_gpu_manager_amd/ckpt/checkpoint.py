"""Asynchronous sharded checkpoints: DeepSpeed file layout, a /dev/shm snapshot tier, agreed restore, resharding.

The reference has no checkpoint code at all; its README claims auto-resume
(``README.md:14``) and its config asks DeepSpeed to gather 16-bit weights on save
(``ai_engine/deepspeed_launcher.py:74, :192``). This module is the MI355X implementation (§2.5 N8).

Capture (training thread, no host sync)
    The rank's fp32 master / exp_avg / exp_avg_sq shards and its bf16 compute shard are copied on a side
    stream into a snapshot buffer: a ``/dev/shm`` file mapped and page-locked (``hipHostRegister``) when the
    host has room ("shm" tier -- it outlives a SIGKILLed rank, so an auto-resume on the same node restores
    from host RAM instead of disk), else spare HBM ("device": D2D at HBM speed) or pinned host memory. The
    next optimizer step waits for the capture *on the GPU* (``stream.wait_event``), so training never
    blocks on the host.
Write-out (background thread)
    Files are real ``torch.save``-format zips (``ckpt/ptzip.py``: pickle generated up front, tensor bytes
    pwritten by the C++ host runtime with 8 threads, CRC32C per 64 MiB chunk for our manifest and the zip
    CRC-32 in the record headers), so ``torch.load(path, weights_only=True)`` reads every one of them::

        <save_dir>/latest                                              "global_step120"
        <save_dir>/global_step120/mp_rank_00_model_states.pt           engine/model metadata, client state
        <save_dir>/global_step120/zero_pp_rank_{r}_mp_rank_00_model_states.pt   rank r's bf16 parameter shard
        <save_dir>/global_step120/zero_pp_rank_{r}_mp_rank_00_optim_states.pt   rank r's fp32 master, exp_avg,
                                                                                exp_avg_sq (DeepSpeed keys)
        <save_dir>/global_step120/manifest_r{r}.json  COMPLETE

    Every save carries a save id (step, restart count, save counter); rank 0 publishes the tag (writes
    ``COMPLETE``, renames ``<tag>.tmp`` -> ``<tag>``, updates ``latest``) only when every writer's manifest
    of THIS save is present, so a manifest left by a crashed earlier attempt cannot publish a half-written tag.
Restore
    Candidates newest first (the shm snapshot when every rank holds the same newest step, then the disk
    tags). Each rank loads and CRC-verifies its part, then all ranks agree (MIN all-reduce of "ok") before
    a candidate is accepted, so no rank can resume from a different step than the others (rollback is
    collective). A world-size or EP-size change reshards: every group is reassembled from the old
    shards -- expert groups expert by expert across the old EP ranks -- and re-sliced for the new layout.
"""
from __future__ import annotations

import hashlib
import json
import math
import os
import queue
import re
import shutil
import threading
import time
from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import _host
from .ptzip import PtWriter, Slot, read_slot
from ..utils.streams import owned_stream

STATE = ("master", "exp_avg", "exp_avg_sq")
TAG_RE = re.compile(r"^global_step(\d+)$")
MODEL0 = "mp_rank_00_model_states.pt"
# the shm snapshot is page-locked in pieces of REG_CHUNK bytes with REG_PAUSE_S between them (_register_chunked):
# 1 GiB pieces with 5 ms pauses kept the first step after a restore at 0.9 s (one whole-file registration: 6.4 s)
REG_CHUNK = 1 << 30
REG_PAUSE_S = 0.005
# background preparation: at most this fraction of the wall time inside hipHostRegister (DLGM_SHM_REG_DUTY)
REG_DUTY = float(os.environ.get("DLGM_SHM_REG_DUTY", "0.3"))
# threads that map each piece (MADV_POPULATE_WRITE, _host.populate_pages) before it is page-locked
MAP_THREADS = 8
# pinned slots of the capture into a not-yet-page-locked part of the shm snapshot (_ring_capture)
RING_SLOT = 256 << 20
RING_SLOTS = 4
DS_VERSION = "0.13.1+dlgm-mi355x"  # the DeepSpeed release the reference pins (requirements.txt:6)


class CorruptCheckpoint(RuntimeError):
    pass


class _ReserveFailed(RuntimeError):
    """posix_fallocate of the shm snapshot failed (tmpfs full): the snapshot moves to the host tier."""


def _tag(step: int) -> str:
    return f"global_step{step}"


def optim_file(rank: int) -> str:
    return f"zero_pp_rank_{rank}_mp_rank_00_optim_states.pt"


def model_file(rank: int) -> str:
    return f"zero_pp_rank_{rank}_mp_rank_00_model_states.pt"


def _layout(eng) -> Dict[str, Any]:
    """What a rank's shard files hold: enough to reassemble every group under any new layout."""
    ep = eng.ep_size
    return {"rank": eng.rank, "world": eng.W, "zero_stage": eng.stage, "ep_size": ep,
            "ep_rank": eng.ep_comm.rank if (ep > 1 and eng.ep_comm is not None) else 0,
            "shard_total": eng.shard_total,
            "groups": [{"name": g.name, "kind": g.kind, "numel": g.numel, "shard_numel": g.shard_numel,
                        "shard_off": g.shard_off, "P": g.P,
                        "prank": (g.comm.rank if g.P > 1 else 0),
                        "params": [[s.name, g.layout[s.name][0], list(s.shape), int(s.experts)] for s in g.specs]}
                       for g in eng.groups]}


def _writer_ranks(eng) -> List[int]:
    """Ranks whose state is not a copy of a lower rank's: every rank under ZeRO-1/2/3; under ZeRO-0 rank 0,
    plus one rank per EP position when experts are split over EP ranks (ranks 0..ep-1)."""
    if eng.stage > 0:
        return list(range(eng.W))
    return list(range(eng.ep_size)) if eng.ep_size > 1 else [0]


def _source_rank(eng) -> int:
    """The writer rank whose files restore this rank (itself, or its ZeRO-0 twin)."""
    if eng.stage > 0:
        return eng.rank
    return eng.rank % eng.ep_size if eng.ep_size > 1 else 0


def shm_snapshot_path(save_dir: str, rank: int) -> str:
    """The /dev/shm snapshot file of `rank` for a job checkpointing into `save_dir` (the checkpointer's and the
    supervisor's shared naming: the supervisor reserves it before the first launch, launcher/supervisor.py)."""
    key = hashlib.sha1(os.path.abspath(save_dir).encode()).hexdigest()[:12]
    return f"/dev/shm/dlgm-ckpt-{key}-r{int(rank)}.snap"


def _prefault(fd: int, lo: int, hi: int, threads: int = 16) -> None:
    """Fault the reserved pages [lo, hi) of a tmpfs file in once, through a throw-away mapping (threaded
    MADV_POPULATE_WRITE): tmpfs zeroes a fallocated page at its first fault, so after this a rank's own mapping only
    builds page tables. Without it the ranks' first touch zeroed 82 GB beside the training loop (the first Mixtral
    step of a fresh job: 5-9 s instead of 1.3-2 s). Best effort: a failure leaves the zeroing to the ranks."""
    import ctypes
    import mmap
    if hi <= lo:
        return
    try:
        mm = mmap.mmap(fd, hi, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
    except (OSError, ValueError):
        return
    try:
        buf = (ctypes.c_char * hi).from_buffer(mm)
        try:
            L = _host.lib()
            if L is not None and hasattr(L, "dlgm_populate_pages"):
                L.dlgm_populate_pages(ctypes.c_void_p(ctypes.addressof(buf) + lo), hi - lo, int(threads), 1)
        finally:
            del buf
    finally:
        mm.close()


def reserve_snapshot_files(save_dir: str, ranks, nbytes: int, threads: int = 8) -> Dict[str, Any]:
    """Reserve (posix_fallocate: tmpfs pages allocated and zeroed) the snapshot file of every rank in `ranks`, at
    least `nbytes` each, WITHOUT touching what a file already holds (a previous attempt's snapshot is the restore
    source): only missing bytes past its current allocation are added. Runs in the supervisor, which outlives the
    ranks, before the first launch: the ranks' own background preparation then finds every page
    reserved and already faulted in once (zeroed, _prefault), and a spot notice at step 1 pays only for mapping and
    page-locking instead of the 3.5-6 GB/s of fresh tmpfs pages. Returns {files, bytes_added, seconds}."""
    import concurrent.futures as cf
    t0 = time.time()
    if not os.path.isdir("/dev/shm") or nbytes <= 0:
        return {"files": [], "bytes_added": 0, "seconds": 0.0, "skipped": "no /dev/shm"}
    st = os.statvfs("/dev/shm")
    jobs = []
    for r in ranks:
        path = shm_snapshot_path(save_dir, r)
        have = 0
        if os.path.exists(path):
            s_ = os.stat(path)
            have = min(s_.st_size, s_.st_blocks * 512)
        if have < nbytes:
            jobs.append((path, have))
    need = sum(nbytes - h for _, h in jobs)
    if need > st.f_bavail * st.f_frsize - (8 << 30):
        return {"files": [p for p, _ in jobs], "bytes_added": 0, "seconds": round(time.time() - t0, 2),
                "skipped": f"/dev/shm too small for {need} B"}
    piece = 1 << 30

    def work(item):
        path, off = item
        fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o600)
        try:
            if os.fstat(fd).st_size < nbytes:
                os.ftruncate(fd, nbytes)
            pieces = [(o, min(piece, nbytes - o)) for o in range(off - off % piece, nbytes, piece)]
            with cf.ThreadPoolExecutor(max(1, threads // max(1, len(jobs)))) as ex:
                list(ex.map(lambda a: os.posix_fallocate(fd, a[0], a[1]), pieces))
            _prefault(fd, off - off % piece, nbytes, max(2, 16 // max(1, len(jobs))))  # ~16 threads in all
        finally:
            os.close(fd)
    with cf.ThreadPoolExecutor(max(1, min(len(jobs), threads))) as ex:
        list(ex.map(work, jobs))
    return {"files": [p for p, _ in jobs], "bytes_added": int(need), "seconds": round(time.time() - t0, 2)}


class _Agree:
    """Cross-rank agreement on small integers (restore decisions), over the engine's communicator."""

    def __init__(self, eng):
        self.comm, self.dev = eng.comm, eng.device

    def min(self, x: float) -> float:
        if self.comm.world == 1:
            return x
        t = torch.tensor([-float(x)], dtype=torch.float64 if self.dev.type == "cpu" else torch.float32,
                         device=self.dev)
        self.comm.all_reduce_max(t)
        return -float(t.item())

    def max(self, x: float) -> float:
        if self.comm.world == 1:
            return x
        t = torch.tensor([float(x)], dtype=torch.float64 if self.dev.type == "cpu" else torch.float32,
                         device=self.dev)
        self.comm.all_reduce_max(t)
        return float(t.item())


class AsyncCheckpointer:
    def __init__(self, engine, save_dir: str, mode: str = "auto", keep_last: int = 3,
                 ring_bytes: int = 1 << 30, manifest_timeout_s: float = 600.0, shm: Any = "auto",
                 disk: bool = True, module: Optional[bool] = None, prepare: bool = True):
        self.engine = eng = engine
        self.save_dir = os.path.abspath(save_dir)
        self.keep_last = keep_last
        self.rank = eng.rank
        self.writers = _writer_ranks(eng)
        self.active = self.rank in self.writers
        self.is_rank0 = eng.rank == 0
        self.n = eng.shard_total
        self.dev = eng.device
        self.cuda = self.dev.type == "cuda"
        self.disk = disk
        self.prepare = prepare  # allocate / page-lock the snapshot buffer in the background before the first save
        self.ring_elems = max(_host.CHUNK // 4, (ring_bytes // 4) // (_host.CHUNK // 4) * (_host.CHUNK // 4))
        self.manifest_timeout_s = manifest_timeout_s
        self.layout = _layout(eng)
        self.sig = hashlib.sha1(json.dumps(self.layout, sort_keys=True).encode()).hexdigest()[:16]
        self.shm_path = shm_snapshot_path(self.save_dir, self.rank)
        self.shm_meta = self.shm_path[:-5] + ".json"
        # restore reads the snapshot of the rank whose files restore this one (a ZeRO-0 twin reads its writer's)
        self.src_rank = _source_rank(eng)
        self.shm_src_path = shm_snapshot_path(self.save_dir, self.src_rank)
        self.shm_src_meta = self.shm_src_path[:-5] + ".json"
        self.tier_notes: List[str] = []
        self.shm_need_bytes = 0
        self.mode = self._pick_mode(mode, shm)
        self._snap: Optional[torch.Tensor] = None  # uint8 [14 n]: fp32 master | exp_avg | exp_avg_sq | bf16 params
        self._pinned_shm = False
        self._reg: List[Tuple[int, int]] = []  # page-locked pieces of the shm snapshot (address, bytes)
        self._falloc_done = 0  # shm snapshot bytes [0, _falloc_done) reserved
        self._mapped_done = 0  # ... [0, _mapped_done) mapped into this process (page tables filled)
        self._reg_done = 0  # ... and [0, _reg_done) page-locked (the DMA part of a save)
        self._reg_failed = False
        self._slots: List[torch.Tensor] = []  # pinned slots of _ring_capture
        self._prep_yield = threading.Event()  # a save needs the buffer now: stop preparing after this piece
        self._reg_stop = threading.Event()
        self._unreg = None
        self._restored_map: Optional[torch.Tensor] = None  # the shm file mapped by a restore (reused, see _load_shm)
        self._ring: List[torch.Tensor] = []
        self._stream = owned_stream(self.dev, "ckpt", owner=self) if self.cuda else None
        self.last_ring: Dict[str, Any] = {}
        self.defer_moments = True  # shm restore: Adam moments restored beside the first step (_load_shm)
        self._moments: Optional[threading.Thread] = None
        self._moments_err: Optional[BaseException] = None
        self._moments_ev = None
        self._capture_ev = None
        self._pending = 0
        self._saves = 0
        self._restart = os.environ.get("DLGM_RESTART", "0")
        self._plock = threading.Lock()
        self._q: "queue.Queue" = queue.Queue()
        self._errors: List[str] = []
        self.history: List[Dict[str, Any]] = []
        self.rollbacks: List[str] = []
        self.restored_from: Optional[str] = None
        self._prep: Optional[threading.Thread] = None
        self.prep_stats: Dict[str, Any] = {}  # snapshot-buffer preparation: fallocate / register seconds
        # the 16-bit module state dict in mp_rank_00_model_states.pt (DeepSpeed: always for stages 0-2; stage 3
        # with stage3_gather_16bit_weights_on_model_save): rank 0 keeps a pinned host copy per save
        self.module = bool(module if module is not None else
                           (eng.stage < 3 or getattr(eng.cfg, "gather_16bit_weights_on_model_save", True)))
        self._mod_snap: Optional[torch.Tensor] = None
        self._mod_index: List[Tuple[str, Tuple[int, ...], int]] = []  # (name, shape, element offset)
        self._touched, self._loaded_meta = False, None
        self._thread = threading.Thread(target=self._writer, daemon=True, name="ckpt-writer")
        self._thread.start()
        eng.pre_step_hooks.append(self._before_optimizer_step)
        os.makedirs(self.save_dir, exist_ok=True)

    # ------------------------------------------------------------------ policy
    @property
    def snap_bytes(self) -> int:
        return 14 * self.n

    def _pick_mode(self, mode: str, shm: Any) -> str:
        if mode in ("device", "host", "shm"):
            return mode
        want_shm = shm is True or (shm == "auto" and self.cuda)
        if want_shm and self._shm_fits():
            if self.active:
                return "shm"
        if not self.active:
            return "host"
        if not self.cuda or getattr(self.engine, "offload", None) is not None:
            return "host"  # offloaded optimizer state already lives in host memory
        free, _ = torch.cuda.mem_get_info(self.dev)
        return "device" if free > self.snap_bytes + (24 << 30) else "host"

    def _shm_fits(self) -> bool:
        """Does /dev/shm hold the snapshots of EVERY writer rank of this node? Collective: the node's need is the
        largest rank snapshot x the local ranks (LOCAL_WORLD_SIZE, torchrun), and the verdict is the minimum over
        all ranks, so every rank picks the same tier (eight Llama-3-70B ranks would need 8 x 123 GB; a per-rank
        check passes on each and overcommits tmpfs together)."""
        agree = _Agree(self.engine)
        need = agree.max(float(self.snap_bytes if self.active else 0)) * max(1, int(os.environ.get(
            "LOCAL_WORLD_SIZE", "1")))
        ok = 0.0
        if os.path.isdir("/dev/shm"):
            st = os.statvfs("/dev/shm")
            ok = 1.0 if st.f_bavail * st.f_frsize > need + (8 << 30) else 0.0
        self.shm_need_bytes = int(need)
        return agree.min(ok) > 0

    def _before_optimizer_step(self, engine) -> None:
        # GPU-side ordering only: the next AdamW must not overwrite master/m/v before the capture read them
        if self._capture_ev is not None and self.cuda:
            torch.cuda.current_stream(self.dev).wait_event(self._capture_ev)

    def _alloc_snapshot(self) -> None:
        t0 = time.time()
        try:
            self._alloc_snapshot_inner()
        finally:
            self.prep_stats["alloc_s"] = round(self.prep_stats.get("alloc_s", 0.0) + time.time() - t0, 2)
            if self.mode != "shm" or self._falloc_done >= self.snap_bytes:
                self.prep_stats["done_at"] = time.time()

    def _alloc_snapshot_inner(self) -> None:
        nb = self.snap_bytes
        if self.mode == "shm":
            if self._snap is None:
                keep, self._restored_map = self._restored_map, None
                if keep is not None and self.shm_path == self.shm_src_path and keep.numel() == nb:
                    self._snap = keep  # the file this rank just restored from, already mapped (pages touched)
                    self._falloc_done = self._mapped_done = nb  # the restore read every page through it
                else:
                    del keep
                    fd = os.open(self.shm_path, os.O_RDWR | os.O_CREAT, 0o600)
                    try:
                        os.ftruncate(fd, nb)
                        if os.fstat(fd).st_blocks * 512 >= nb:
                            # every page already reserved (the supervisor's reserve_snapshot_files, or a previous
                            # attempt's file): the preparation only maps and page-locks
                            self._falloc_done = nb
                            self.prep_stats["pre_reserved"] = True
                    finally:
                        os.close(fd)
                    self._snap = torch.from_file(self.shm_path, shared=True, size=nb, dtype=torch.uint8)
            if not self._prepare_shm(nb):
                try:
                    os.unlink(self.shm_path)
                except OSError:
                    pass
                self.mode = "host"
                self._snap = torch.empty(nb, dtype=torch.uint8, pin_memory=self.cuda)
        elif self.mode == "device":
            self._snap = torch.empty(nb, dtype=torch.uint8, device=self.dev)
            self._ring = [torch.empty(self.ring_elems, dtype=torch.float32, pin_memory=True) for _ in range(2)]
        else:
            self._snap = torch.empty(nb, dtype=torch.uint8, pin_memory=self.cuda)

    @staticmethod
    def _hip_register_fns():
        """(register, unregister) through ctypes on the HIP runtime torch already loaded: a ctypes foreign call
        releases the GIL, so page-locking ~100 GB on a background thread does not stall the training loop's
        Python thread (torch.cuda.cudart() holds the GIL for the whole call)."""
        import ctypes
        try:
            lib = ctypes.CDLL("libamdhip64.so")
        except OSError:
            return None
        reg, unreg = lib.hipHostRegister, lib.hipHostUnregister
        reg.restype, reg.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
        unreg.restype, unreg.argtypes = ctypes.c_int, [ctypes.c_void_p]
        return (lambda p_, n_: int(reg(p_, n_, 0))), (lambda p_: int(unreg(p_)))

    def _prepare_shm(self, nb: int) -> bool:
        """Make the mapped snapshot file ready for a DMA capture in the background: _ready_pipeline with a short
        pause between page-locked pieces (one hipHostRegister of a whole ~112 GB file holds the HIP runtime for ~6 s
        and every kernel launch of the training thread waits meanwhile; MI355X: the first step after a restore took
        6.4 s instead of 0.9 s). The page-locked prefix [0, _reg_done) is what a save copies by DMA at ~57 GB/s; a
        save that arrives first (an early spot notice) sets _prep_yield, the pipeline stops after its current
        pieces, and the save runs the same pipeline for the rest itself (_lock_and_dma). Returns False when the
        reservation failed (the caller falls back to the host tier)."""
        def stopped() -> bool:
            return self._prep_yield.is_set() or self._reg_stop.is_set()
        t0 = time.time()
        try:
            self._ready_pipeline(nb, stop=stopped, pause=REG_PAUSE_S)
        except _ReserveFailed:
            self._unregister_all()
            return False
        finally:
            self.prep_stats["pipeline_s"] = round(self.prep_stats.get("pipeline_s", 0.0) + time.time() - t0, 3)
        return True

    def _ready_pipeline(self, hi: int, stop=None, pause: float = 0.0, on_locked=None) -> int:
        """Snapshot pieces [_reg_done, hi) of REG_CHUNK bytes through three stages that run concurrently, one piece
        apart: a thread reserves (posix_fallocate: a full tmpfs is an error here, not a SIGBUS in a later copy),
        a thread maps the pages (inside a save: writable, MADV_POPULATE_WRITE on MAP_THREADS threads; in the
        background preparation, or where that is unavailable: one byte read per page, which leaves the training
        loop alone), and the calling thread page-locks (hipHostRegister), then calls on_locked(off, ln). On
        the MI355X host, 24 GiB each: reserve 17-19.5 GB/s; map 64 GB/s by populate-write on 8-16 threads against
        13-16 GB/s by touching (on any number of threads); page-lock 118-133 GB/s for populate-written pages, 37-41
        for read-touched ones, 12.6 for reserved-but-unmapped ones (profiles/shm_map_bench_r05.json, _r06.json) -- so
        a supervisor-reserved file is mapped and locked at ~40 GB/s. Without a GPU it only reserves. Returns the end
        of the page-locked range (< hi after a stop or a failed registration: the rest then goes through the pinned
        slots)."""
        fns = self._hip_register_fns() if self.cuda else None
        if self.cuda and fns is None:
            cr = torch.cuda.cudart()
            fns = (lambda p_, n_: int(cr.cudaHostRegister(p_, n_, 0))), (lambda p_: int(cr.cudaHostUnregister(p_)))
        if fns is not None:
            self._unreg = fns[1]
        halt = threading.Event()
        err: List[str] = []

        def reserve():
            fd = os.open(self.shm_path, os.O_RDWR)
            try:
                while self._falloc_done < hi and not halt.is_set():
                    tf = time.time()
                    if not self._reserve(fd, self._falloc_done, min(REG_CHUNK, hi - self._falloc_done)):
                        err.append(self.tier_notes[-1])
                        return
                    self.prep_stats["fallocate_s"] = round(self.prep_stats.get("fallocate_s", 0.0) + time.time() - tf, 3)
            finally:
                os.close(fd)

        def map_pages():
            while self._mapped_done < hi and not halt.is_set() and not err:
                off = self._mapped_done
                ln = min(REG_CHUNK, hi - off)
                if self._falloc_done < off + ln:
                    time.sleep(0.0005)
                    continue
                piece = self._snap[off:off + ln]
                # a save maps with MADV_POPULATE_WRITE on threads (64 GB/s); the background preparation touches one
                # byte per page instead: populate threads running beside the training loop held the first Mixtral
                # step at 5-9 s (touching: 1.3 s), profiles/drills_mixtral_8x7b_ep8_shadow_r06.json "map_ab"
                mode = os.environ.get("DLGM_SHM_MAP") or ("touch" if pause > 0 else "write")
                if mode == "touch" or not _host.populate_pages(piece, MAP_THREADS, write=mode != "read"):
                    int(piece[::4096].sum())  # one byte per page: map it (13-16 GB/s on one or more threads)
                self._mapped_done = off + ln

        ths = [threading.Thread(target=reserve, daemon=True, name="ckpt-reserve")]
        if fns is not None and not self._reg_failed:
            ths.append(threading.Thread(target=map_pages, daemon=True, name="ckpt-map"))
        for t in ths:
            t.start()
        ptr, off = self._snap.data_ptr(), self._reg_done
        try:
            if fns is None or self._reg_failed:
                while self._falloc_done < hi and not err and not (stop and stop()):
                    time.sleep(0.001)
            else:
                while off < hi:
                    if stop is not None and stop():
                        break
                    ln = min(REG_CHUNK, hi - off)
                    if self._mapped_done < off + ln and not err:
                        time.sleep(0.0005)
                        continue
                    if err:
                        break
                    tr = time.time()
                    if fns[0](ptr + off, ln) != 0:
                        self._reg_failed = True  # the rest goes through the pinned slots; never a correctness issue
                        self.tier_notes.append("hipHostRegister of the shm snapshot failed; pinned-slot capture")
                        break
                    self._reg.append((ptr + off, ln))
                    self._reg_done = off + ln
                    dt = time.time() - tr
                    self.prep_stats["register_s"] = round(self.prep_stats.get("register_s", 0.0) + dt, 3)
                    if on_locked is not None:
                        on_locked(off, ln)
                    off += ln
                    if pause > 0 and off < hi:
                        # background preparation: hipHostRegister holds the HIP runtime, so the training thread's
                        # launches wait while it runs -- keep it to REG_DUTY of the wall time (with populate-written
                        # pages a 1 GiB piece locks in ~8 ms; back to back they held the first Mixtral step at 5.9 s)
                        time.sleep(max(pause, dt * (1.0 / REG_DUTY - 1.0)))
        finally:
            halt.set()
            for t in ths:
                t.join()
        if err:
            raise _ReserveFailed(err[0])
        self._pinned_shm = self.cuda and self._reg_done >= self.snap_bytes
        return off

    def _reserve(self, fd: int, off: int, ln: int) -> bool:
        """posix_fallocate one piece of the snapshot file (the next unreserved one)."""
        try:
            os.posix_fallocate(fd, off, ln)
        except OSError as e:
            self.tier_notes.append(f"shm reservation of {self.snap_bytes} B failed ({e}); snapshot tier -> host memory")
            return False
        self._falloc_done = off + ln
        return True

    def _unregister_all(self) -> None:
        if self._unreg is not None:
            for p_, _ in self._reg:
                self._unreg(p_)
        self._reg, self._reg_done, self._pinned_shm = [], 0, False

    def _copy_to_snap(self, dst: torch.Tensor, src: torch.Tensor) -> None:
        """dst (a flat view of the snapshot) <- src, asynchronously, never crossing a page-locked piece."""
        if not self._reg:
            dst.copy_(src, non_blocking=True)
            return
        es, n = dst.element_size(), dst.numel()
        base = dst.data_ptr() - self._snap.data_ptr()
        i = 0
        while i < n:
            b = base + i * es
            m = min(n - i, ((b // REG_CHUNK + 1) * REG_CHUNK - b) // es)
            dst[i:i + m].copy_(src[i:i + m], non_blocking=True)
            i += m

    def _ring_capture(self, segs: List[Tuple[int, torch.Tensor]], lo: int, hi: int) -> List[int]:
        """Snapshot bytes [lo, hi) <- the device state, through RING_SLOTS pinned slots: the D2H of piece k+1..
        runs on the checkpoint stream while _host's 16 threads copy piece k into the mapping with the per-CHUNK
        CRC32C of the copied bytes. Blocks the calling thread; ~31 GB/s on MI355X into reserved pages against
        ~9 GB/s for a plain copy into an unregistered mapping (tools/diag/r05/shm_bench.py). Pages the preparation
        has not reserved yet are reserved by a helper thread running ahead of the copy (posix_fallocate ~19 GB/s;
        letting the copy fault them in ran at 3.8 GB/s). `segs`: (snapshot byte offset, flat uint8 view of the
        device source). lo is CHUNK-aligned."""
        if not self._slots:
            ta = time.time()
            self._slots = [torch.empty(RING_SLOT, dtype=torch.uint8, pin_memory=True) for _ in range(RING_SLOTS)]
            self.last_ring["slots_alloc_s"] = round(time.time() - ta, 3)
        crcs: List[int] = []
        pend: List[Tuple[int, int, int, Any]] = []
        res_err: List[str] = []
        resv = None
        if self.mode == "shm" and self._falloc_done < hi:
            def reserve_ahead():
                fd = os.open(self.shm_path, os.O_RDWR)
                try:
                    while self._falloc_done < hi:
                        if not self._reserve(fd, self._falloc_done, min(REG_CHUNK, hi - self._falloc_done)):
                            res_err.append(self.tier_notes[-1])
                            return
                finally:
                    os.close(fd)
            resv = threading.Thread(target=reserve_ahead, daemon=True, name="ckpt-reserve")
            resv.start()

        tw = {"wait_reserve_s": 0.0, "wait_d2h_s": 0.0, "copy_s": 0.0}

        def drain():
            k, off, ln, ev = pend.pop(0)
            t0 = time.time()
            while self._falloc_done < off + ln and not res_err:
                time.sleep(0.0005)
            if res_err:
                raise _ReserveFailed(res_err[0])
            t1 = time.time()
            ev.synchronize()
            t2 = time.time()
            crcs.extend(_host.copy_crc32c_chunks(self._slots[k % RING_SLOTS][:ln], self._snap[off:off + ln]))
            tw["wait_reserve_s"] += t1 - t0
            tw["wait_d2h_s"] += t2 - t1
            tw["copy_s"] += time.time() - t2
        try:
            for k, off in enumerate(range(lo, hi, RING_SLOT)):
                if len(pend) == RING_SLOTS:
                    drain()
                ln = min(RING_SLOT, hi - off)
                slot = self._slots[k % RING_SLOTS]
                with torch.cuda.stream(self._stream):
                    for base, src in segs:
                        a, b = max(off, base), min(off + ln, base + src.numel())
                        if a < b:
                            slot[a - off:b - off].copy_(src[a - base:b - base], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self._stream)
                pend.append((k, off, ln, ev))
            while pend:
                drain()
        finally:
            if resv is not None:
                resv.join()
        self.last_ring.update({k: round(v, 3) for k, v in tw.items()})
        return crcs

    def _lock_and_dma(self, segs: List[Tuple[int, torch.Tensor]], lo: int, hi: int) -> int:
        """Finish the preparation inside a save that came first: _ready_pipeline over [lo, hi) without pauses, each
        piece's D2H queued on the checkpoint stream as soon as it is page-locked (the DMA of piece k runs while
        piece k+1 is being reserved / mapped / locked). The first versions measured what this avoids: a pinned-slot
        copy into a fresh mapping, or page-locking unmapped pages, both ran at ~5 GB/s inside the trainer (Mixtral
        EP = 8 spot drill, 81.7 GB: 17.1 s / 15.4 s). Returns the end of the locked range. `segs`: (snapshot offset,
        uint8 device view)."""
        def dma(off: int, ln: int) -> None:
            with torch.cuda.stream(self._stream):
                for base, src in segs:
                    a, b = max(off, base), min(off + ln, base + src.numel())
                    if a < b:
                        self._snap[a:b].copy_(src[a - base:b - base], non_blocking=True)
        return self._ready_pipeline(hi, on_locked=dma)  # _ReserveFailed: save() falls back to the host tier

    def prepare_async(self) -> None:
        """Reserve (and page-lock) the snapshot buffer on a background thread while training runs, so the
        first save -- often an emergency one on a spot notice -- does not pay for 14 B/param of fresh host
        pages. Called when the job starts (and again after a save that interrupted it)."""
        if not self.prepare:
            return
        if self.active and self._prep is None and (self._snap is None or (
                self.mode == "shm" and (self._falloc_done < self.snap_bytes or
                                        (self.cuda and not self._reg_failed and self._reg_done < self.snap_bytes)))):
            self.prep_stats.setdefault("started_at", time.time())
            self._prep = threading.Thread(target=self._alloc_snapshot, daemon=True, name="ckpt-prepare")
            self._prep.start()

    def _views(self, snap: torch.Tensor) -> Dict[str, torch.Tensor]:
        n = self.n
        f = snap[:12 * n].view(torch.float32).view(3, n)
        # "bf16": the 16-bit compute copy (fp16 when the engine runs the fp16 path)
        return {"master": f[0], "exp_avg": f[1], "exp_avg_sq": f[2],
                "bf16": snap[12 * n:14 * n].view(self.engine.p16_shard.dtype)}

    # ------------------------------------------------------------------ save
    def _capture_device(self, srcs) -> Optional[Tuple[int, List[int]]]:
        """Queue the D2H capture of `srcs` (snapshot view, device tensor) on the checkpoint stream. shm tier: the
        page-locked prefix by DMA; a save that came before the preparation finished page-locks the rest itself,
        piece by piece, each piece's DMA queued as soon as it is locked (_lock_and_dma); anything that could not be
        locked goes through the pinned slots (the returned CRCs). Raises _ReserveFailed when the rest of the shm file
        cannot be reserved."""
        dma_end = self._reg_done if (self.mode == "shm" and not self._pinned_shm) else self.snap_bytes
        with torch.cuda.stream(self._stream):
            for dst, s in srcs:
                a = dst.data_ptr() - self._snap.data_ptr()
                n_dma = max(0, min(dst.numel() * dst.element_size(), dma_end - a)) // dst.element_size()
                if n_dma:
                    self._copy_to_snap(dst[:n_dma], s[:n_dma])
        if dma_end >= self.snap_bytes:
            return None
        segs = [(dst.data_ptr() - self._snap.data_ptr(), s.reshape(-1).view(torch.uint8)) for dst, s in srcs]
        tr = time.time()
        locked = self._lock_and_dma(segs, dma_end, self.snap_bytes) if not self._reg_failed else dma_end
        self.last_ring.update(locked_bytes=locked - dma_end, lock_s=round(time.time() - tr, 3))
        if locked >= self.snap_bytes:
            return None
        tr = time.time()
        crcs = (locked, self._ring_capture(segs, locked, self.snap_bytes))
        self.last_ring.update(bytes=self.snap_bytes - locked, s=round(time.time() - tr, 3))
        return crcs

    def _fall_back_to_host(self, why: str) -> None:
        """shm tier -> pinned host tier inside a save: the DMAs already queued into the mapping finish before its
        pages are unlocked and the file is dropped."""
        self._stream.synchronize()
        self._unregister_all()
        self.tier_notes.append(f"shm snapshot failed during a save ({why}); snapshot tier -> host memory")
        self.last_ring["fell_back_to_host"] = why
        try:
            os.unlink(self.shm_path)
        except OSError:
            pass
        self.mode = "host"
        self._snap = torch.empty(self.snap_bytes, dtype=torch.uint8, pin_memory=self.cuda)

    def save(self, step: int, client_state: Optional[Dict[str, Any]] = None, blocking: bool = False) -> str:
        t0 = time.time()
        tag = _tag(step)
        self._saves += 1
        if not self.active:
            return tag
        self.engine.join_optimizer()  # an overlapped optimizer update may still be writing the state
        self._await_moments()  # a deferred restore still reading the snapshot file this save overwrites
        if self.busy:  # previous write-out still streaming from the snapshot buffer
            self.wait()
        save_id = f"{step}.{self._restart}.{self._saves}"
        interrupted = False
        self.last_ring = {}
        if self._prep is not None:
            tj = time.time()
            self._prep_yield.set()  # a save is waiting: stop preparing after the current piece
            self._prep.join()
            self._prep = None
            self._prep_yield.clear()
            interrupted = True
            self.last_ring = {"prep_join_s": round(time.time() - tj, 3)}
        if self._snap is None or (not self.prepare and self.mode == "shm" and self._falloc_done < self.snap_bytes):
            self._alloc_snapshot()
        if self.mode == "shm" and os.path.exists(self.shm_meta):
            os.unlink(self.shm_meta)  # the snapshot is about to change: never restore a torn one
        eng = self.engine
        v = self._views(self._snap)
        srcs = [(v["master"], eng.master), (v["exp_avg"], eng.exp_avg), (v["exp_avg_sq"], eng.exp_avg_sq),
                (v["bf16"], eng.p16_shard)]
        ring_crcs: Optional[Tuple[int, List[int]]] = None
        if self.cuda:
            cur = torch.cuda.current_stream(self.dev)
            self._stream.wait_stream(cur)
            try:
                ring_crcs = self._capture_device(srcs)
            except _ReserveFailed as e:
                # the tmpfs filled up while this save reserved the rest of the snapshot file (an early spot notice
                # that interrupted the background preparation): the emergency checkpoint must still happen, so the
                # state goes to a pinned host buffer instead, the way _alloc_snapshot falls back
                self._fall_back_to_host(str(e))
                v = self._views(self._snap)
                srcs = [(v["master"], eng.master), (v["exp_avg"], eng.exp_avg), (v["exp_avg_sq"], eng.exp_avg_sq),
                        (v["bf16"], eng.p16_shard)]
                ring_crcs = self._capture_device(srcs)
            with torch.cuda.stream(self._stream):
                ev = torch.cuda.Event()
                ev.record(self._stream)
            self._capture_ev = ev
        else:
            for dst, s in srcs:
                dst.copy_(s)
            ev = None
        if interrupted:
            self.prepare_async()  # page-lock the rest in the background for the next save
        mod_ev = self._capture_module() if (self.module and self.disk) else None
        meta = self._meta(step, client_state or {})
        meta["_module_ev"] = mod_ev
        meta["_ring_crcs"] = ring_crcs
        meta["_capture_notes"] = dict(self.last_ring)
        with self._plock:
            self._pending += 1
        self._q.put((tag, step, save_id, ev, meta, t0))
        if blocking:
            self.wait()
        return tag

    def _capture_module(self):
        """Gather the 16-bit parameters group by group (a collective on every rank: ZeRO shards and EP experts)
        and copy them, on rank 0, into a pinned host buffer on the snapshot stream. Returns what the writer
        waits for before streaming the module into mp_rank_00_model_states.pt (True on CPU)."""
        eng = self.engine
        dt = eng.p16_shard.dtype
        if self.is_rank0 and self._mod_snap is None:
            off, idx = 0, []
            for name, shp in eng.module_shapes():
                idx.append((name, shp, off))
                off += math.prod(shp)
            self._mod_index = idx
            self._mod_snap = torch.empty(off, dtype=dt, pin_memory=self.cuda)
        pos = {n: (shp, o) for n, shp, o in self._mod_index}
        cur = torch.cuda.current_stream(self.dev) if self.cuda else None
        for items in eng.iter_full(eng.master, dt):
            if not self.is_rank0:
                continue
            for name, t in items:
                shp, o = pos[name]
                dst = self._mod_snap[o:o + t.numel()]
                if self.cuda:
                    self._stream.wait_stream(cur)
                    with torch.cuda.stream(self._stream):
                        dst.copy_(t.reshape(-1), non_blocking=True)
                    t.record_stream(self._stream)
                else:
                    dst.copy_(t.reshape(-1))
        if not self.is_rank0:
            return None
        if not self.cuda:
            return True
        ev = torch.cuda.Event()
        ev.record(self._stream)
        return ev

    def _write_model0(self, path: str, meta: Dict[str, Any], mod_ev) -> None:
        meta = {k: v for k, v in meta.items() if k != "_module_ev"}
        if mod_ev is None or self._mod_snap is None:
            torch.save(meta, path)
            return
        if mod_ev is not True:
            while not mod_ev.query():
                time.sleep(0.0005)
        dt = self._mod_snap.dtype
        meta["module"] = {name: Slot("module/" + name, dt, shp) for name, shp, _ in self._mod_index}
        w = PtWriter(path, meta)
        for name, shp, o in self._mod_index:
            self._stream_host(w, "module/" + name, self._mod_snap[o:o + math.prod(shp)])
        w.close(fsync=True)

    def _stream_host(self, w: PtWriter, name: str, src: torch.Tensor) -> None:
        """Write a host tensor into slot `name` in ring-sized pieces."""
        per = self.ring_elems * 4 // src.element_size()
        for off in range(0, src.numel(), per):
            w.write(name, src[off:off + per], off * src.element_size())

    def _meta(self, step: int, client_state: Dict[str, Any]) -> Dict[str, Any]:
        eng = self.engine
        ecfg = {k: (str(v) if isinstance(v, torch.dtype) else list(v) if isinstance(v, tuple) else v)
                for k, v in vars(eng.cfg).items()}
        groups = [{"name": g.name, "prefix": g.prefix, "numel": g.numel, "shard_numel": g.shard_numel,
                   "shard_off": g.shard_off, "kind": g.kind,
                   "params": [[s.name, g.layout[s.name][0], list(s.shape)] for s in g.specs]}
                  for g in eng.groups]
        return {"ds_version": DS_VERSION, "global_steps": step, "global_samples": step * eng.cfg.micro_batch_size
                * eng.cfg.grad_accum * eng.W, "dp_world_size": eng.W, "mp_world_size": 1,
                "partition_count": eng.P, "zero_stage": eng.stage, "ep_size": eng.ep_size,
                "model_config": eng.mcfg.to_dict(), "engine_config": ecfg, "groups": groups, "writers": self.writers,
                "client_state": client_state, "lr_scheduler": {"last_batch_iteration": step},
                "param_shapes": [{f"{g['prefix']}.{p[0]}": p[2] for p in g["params"]} for g in groups],
                "buffer_names": [], "module": None,
                # DeepSpeed keeps the scaler in the checkpoint; restore resumes at the saved scale and counters
                "loss_scaler": (eng.scaler.state_dict() if eng.scaler is not None else None)}

    @property
    def prepared(self) -> bool:
        """The snapshot buffer is ready for a capture at DMA rate: nothing is left for the background preparation
        (reserved and, with a GPU, page-locked -- or the page-locking failed and the pinned slots carry it)."""
        if not self.active:
            return True
        if self._snap is None:
            return False
        if self.mode != "shm":
            return True
        if self._falloc_done < self.snap_bytes:
            return False
        return not self.cuda or self._reg_failed or self._reg_done >= self.snap_bytes

    @property
    def busy(self) -> bool:
        with self._plock:
            return self._pending > 0

    def wait(self, timeout_s: float = 3600.0) -> None:
        t0 = time.time()
        while self.busy and time.time() - t0 < timeout_s:
            time.sleep(0.005)
        if self._errors:
            raise RuntimeError("checkpoint write failed: " + "; ".join(self._errors))

    def wait_published(self, step: int, timeout_s: float = 600.0) -> bool:
        """Block until tag `step` is complete on disk (published by rank 0) -- fault drills kill after this."""
        t0 = time.time()
        while time.time() - t0 < timeout_s:
            if os.path.exists(os.path.join(self.save_dir, _tag(step), "COMPLETE")) or not self.disk:
                return True
            time.sleep(0.01)
        return False

    def _writer(self) -> None:
        while True:
            job = self._q.get()
            try:
                self._write_one(*job)
            except Exception as e:  # noqa: BLE001
                self._errors.append(f"{job[0]}: {type(e).__name__}: {e}")
            finally:
                with self._plock:
                    self._pending -= 1

    def _host_piece(self, src: torch.Tensor, off: int, ln: int, k: int) -> torch.Tensor:
        """Elements [off, off+ln) of snapshot tensor `src` as a contiguous CPU tensor (device mode: via the ring)."""
        if self.mode != "device":
            return src[off:off + ln]
        slot = self._ring[k % 2].view(torch.uint8)[:ln * src.element_size()].view(src.dtype)
        with torch.cuda.stream(self._stream):
            slot.copy_(src[off:off + ln], non_blocking=True)
            e2 = torch.cuda.Event()
            e2.record(self._stream)
        e2.synchronize()  # this background thread only
        return slot

    def _stream_slot(self, w: PtWriter, name: str, src: torch.Tensor) -> None:
        per = self.ring_elems * 4 // src.element_size()
        for k, off in enumerate(range(0, src.numel(), per)):
            ln = min(per, src.numel() - off)
            w.write(name, self._host_piece(src, off, ln, k), off * src.element_size())

    def _write_one(self, tag: str, step: int, save_id: str, ev, meta: Dict[str, Any], t0: float) -> None:
        if ev is not None:
            while not ev.query():
                time.sleep(0.0005)
        t_cap = time.time()
        v = self._views(self._snap)
        ring_crcs = meta.pop("_ring_crcs", None)
        notes = meta.pop("_capture_notes", None)
        rec: Dict[str, Any] = {"tag": tag, "step": step, "capture_s": t_cap - t0, "mode": self.mode,
                               "bytes": self.snap_bytes}
        if notes:
            rec["ring"] = notes
        if self.mode == "shm":
            if ring_crcs is not None:  # the pinned-slot part was checksummed while it was copied
                lo, tail = ring_crcs
                crcs = (_host.crc32c_chunks(self._snap[:lo]) if lo else []) + list(tail)
            else:
                crcs = _host.crc32c_chunks(self._snap)
            tmpm = self.shm_meta + ".tmp"
            with open(tmpm, "w") as f:
                json.dump({"save_dir": self.save_dir, "step": step, "save_id": save_id, "sig": self.sig,
                           "bytes": self.snap_bytes, "crc": crcs, "algo": _host.algo(),
                           "meta": {k: v for k, v in meta.items() if k != "_module_ev"}}, f)
            os.replace(tmpm, self.shm_meta)
            if os.path.exists(self.shm_meta + ".bad"):  # a fresh snapshot replaces one a restore found bad
                os.unlink(self.shm_meta + ".bad")
            rec["shm_s"] = time.time() - t_cap
        if not self.disk:
            self.history.append(rec)
            return
        tmp = os.path.join(self.save_dir, tag + ".tmp")
        os.makedirs(tmp, exist_ok=True)
        eng = self.engine
        lay = self.layout
        files: Dict[str, Dict[str, Any]] = {}
        # optimizer states: DeepSpeed's ZeRO keys (fp32_flat_groups + the Adam state of the flat group)
        optim = {"optimizer_state_dict": {
            "zero_stage": eng.stage, "partition_count": eng.P, "loss_scaler": meta["loss_scaler"],
            "dynamic_loss_scale": eng.scaler is not None and eng.scaler.dynamic, "overflow": False,
            "fp32_flat_groups": [Slot("master", torch.float32, (self.n,))],
            "optimizer_state_dict": {"state": {0: {"step": step, "exp_avg": Slot("exp_avg", torch.float32, (self.n,)),
                                                   "exp_avg_sq": Slot("exp_avg_sq", torch.float32, (self.n,))}},
                                     "param_groups": [{"lr": None, "betas": list(eng.cfg.betas), "eps": eng.cfg.eps,
                                                       "weight_decay": eng.cfg.weight_decay, "params": [0]}]}},
            "ds_config": meta["engine_config"], "ds_version": DS_VERSION, "dlgm_layout": lay}
        path = os.path.join(tmp, optim_file(self.rank))
        w = PtWriter(path, optim)
        for name in STATE:
            self._stream_slot(w, name, v[name])
        files[optim_file(self.rank)] = w.close(fsync=True)
        model = {"module": {}, "buffer_names": [], "param_shapes": meta["param_shapes"],
                 "bf16_param_shard": Slot("bf16", eng.p16_shard.dtype, (self.n,)), "ds_version": DS_VERSION,
                 "global_steps": step, "dp_world_size": eng.W, "mp_world_size": 1, "dlgm_layout": lay}
        path = os.path.join(tmp, model_file(self.rank))
        w = PtWriter(path, model)
        self._stream_slot(w, "bf16", v["bf16"])
        files[model_file(self.rank)] = w.close(fsync=True)
        if self.is_rank0:
            self._write_model0(os.path.join(tmp, MODEL0), meta, meta.get("_module_ev"))
        man = {"rank": self.rank, "save_id": save_id, "step": step, "layout": lay, "files": files}
        mtmp = os.path.join(tmp, f".manifest_r{self.rank}.json")
        with open(mtmp, "w") as f:
            json.dump(man, f)
        os.replace(mtmp, os.path.join(tmp, f"manifest_r{self.rank}.json"))
        rec["write_s"] = time.time() - t_cap
        if self.is_rank0:
            self._publish(tag, tmp, step, save_id)
            rec["published_s"] = time.time() - t0
        self.history.append(rec)

    def _publish(self, tag: str, tmp: str, step: int, save_id: str) -> None:
        deadline = time.time() + self.manifest_timeout_s
        while time.time() < deadline:
            ok = True
            for r in self.writers:
                p = os.path.join(tmp, f"manifest_r{r}.json")
                try:
                    with open(p) as f:
                        ok = ok and json.load(f).get("save_id") == save_id
                except (OSError, ValueError):
                    ok = False
                if not ok:
                    break
            if ok:
                break
            time.sleep(0.05)
        else:
            raise TimeoutError(f"{tag}: not every rank wrote its manifest for save {save_id}")
        open(os.path.join(tmp, "COMPLETE"), "w").write(str(step))
        final = os.path.join(self.save_dir, tag)
        if os.path.exists(final):
            shutil.rmtree(final)
        os.replace(tmp, final)
        ltmp = os.path.join(self.save_dir, ".latest.tmp")
        with open(ltmp, "w") as f:
            f.write(tag)
        os.replace(ltmp, os.path.join(self.save_dir, "latest"))
        self._prune()

    def _prune(self) -> None:
        tags = complete_tags(self.save_dir)
        for t in tags[:-self.keep_last] if self.keep_last > 0 else []:
            shutil.rmtree(os.path.join(self.save_dir, t), ignore_errors=True)

    # ------------------------------------------------------------------ restore
    def _shm_step(self) -> int:
        if os.path.exists(self.shm_src_meta + ".bad"):
            return -1
        try:
            with open(self.shm_src_meta) as f:
                m = json.load(f)
            if m.get("save_dir") == self.save_dir and m.get("sig") == self._src_sig() and \
                    os.path.getsize(self.shm_src_path) >= m["bytes"]:
                return int(m["step"])
        except (OSError, ValueError, KeyError):
            pass
        return -1

    def load(self, tag: str = "auto", verify: bool = True) -> Optional[Dict[str, Any]]:
        """Restore engine state; returns the client state (None when no checkpoint exists). Collective.

        ``tag="auto"``: the newest candidate that loads and verifies on EVERY rank -- the shm snapshot tier
        when all ranks hold the same newest step, else the disk tags newest first; a candidate that fails
        on any rank is rolled back on all of them (recorded in ``self.rollbacks``)."""
        self.rollbacks = []
        self.engine.join_optimizer()
        self._await_moments()
        self.restore_stats: Dict[str, Any] = {}
        agree = _Agree(self.engine)
        auto = tag in ("auto", "latest")
        disk = list(reversed(complete_tags(self.save_dir))) if auto else [tag]
        newest_disk = int(TAG_RE.match(disk[0]).group(1)) if disk and TAG_RE.match(disk[0]) else -1
        cands: List[Tuple[str, str]] = []
        if auto:
            s = self._shm_step()
            lo, hi = agree.min(s), agree.max(s)
            if lo >= 0 and lo == hi and lo >= newest_disk:
                cands.append(("shm", _tag(int(lo))))
        cands += [("disk", t) for t in disk]
        touched = False  # some candidate wrote into the engine's state before failing
        for kind, t in cands:
            err = ""
            cs: Optional[Dict[str, Any]] = None
            t0 = time.time()
            self._touched, self._loaded_meta = False, None
            try:
                cs = self._load_shm() if kind == "shm" else self._load_tag(t, verify)
            except (CorruptCheckpoint, FileNotFoundError, OSError, KeyError, ValueError, RuntimeError) as e:
                err = f"{type(e).__name__}: {e}"
            touched = touched or self._touched
            t1 = time.time()
            if agree.min(0.0 if err else 1.0) > 0:
                t2 = time.time()
                ls = (self._loaded_meta or {}).get("loss_scaler")
                if self.engine.scaler is not None and isinstance(ls, dict) and "cur_scale" in ls:
                    self.engine.scaler.load_state_dict(ls)
                self.engine.sync_params_from_master()
                if self.cuda:
                    torch.cuda.synchronize(self.dev)
                self.restore_stats.update(read_s=round(t1 - t0, 2), agree_s=round(t2 - t1, 2),
                                          params_s=round(time.time() - t2, 2))
                self.restored_from = f"{kind}:{t}"
                return cs
            self.rollbacks.append(f"{kind}:{t}: {err or 'failed on another rank'}")
            if not auto:
                raise CorruptCheckpoint(f"{t}: {err or 'failed on another rank'}")
        if agree.max(1.0 if touched else 0.0) > 0:
            # a candidate failed part-way through overwriting the optimizer state and no later one replaced
            # it: the engine holds a mix of checkpoints, never something to train on (or to start from step 0)
            raise CorruptCheckpoint("every checkpoint candidate failed after a partial restore: "
                                    + "; ".join(self.rollbacks))
        return None

    def _src_sig(self) -> str:
        lay = dict(self.layout, rank=self.src_rank)
        return hashlib.sha1(json.dumps(lay, sort_keys=True).encode()).hexdigest()[:16]

    def _load_shm(self) -> Dict[str, Any]:
        """Restore from the /dev/shm snapshot: the file is memory-mapped and CHUNK-aligned pieces are copied into
        two pinned slots by 16 C++ threads (CRC32C of the copied bytes on the fly); each piece goes on to the
        fp32 state on the device while the next one is copied. Copying through the mapping touches the
        never-read shared pages at ~90 GB/s on an MI355X host where pread of them ran at ~16 GB/s
        (tools/diag/shm_read_bench.cpp)."""
        with open(self.shm_src_meta) as f:
            m = json.load(f)
        eng, n = self.engine, self.n
        dsts = [(k * 4 * n, getattr(eng, name).view(torch.uint8)) for k, name in enumerate(STATE)]
        end = 12 * n  # the bf16 copy after the fp32 state is recomputed from the master, not read
        piece = max(_host.CHUNK, self.ring_elems * 4)
        check = m["algo"] == _host.algo()
        ta = time.time()
        slots = [torch.empty(piece, dtype=torch.uint8, pin_memory=self.cuda) for _ in range(2)]
        self.restore_stats["pin_s"] = round(time.time() - ta, 2)
        waited = [0.0, 0.0]  # [main thread waiting for a read, waiting for an H2D]
        jobs = [(k, off, min(piece, end - off)) for k, off in enumerate(range(0, end, piece))]
        q: "queue.Queue" = queue.Queue(maxsize=1)
        free = [threading.Semaphore(1), threading.Semaphore(1)]
        stop = threading.Event()  # set when the main loop gives up: the reader must not block forever

        tm = time.time()
        fmap = torch.from_file(self.shm_src_path, shared=True, size=os.path.getsize(self.shm_src_path),
                               dtype=torch.uint8) if _host.lib() is not None else None
        self.restore_stats["map_s"] = round(time.time() - tm, 2)

        def put(item) -> bool:
            while not stop.is_set():
                try:
                    q.put(item, timeout=0.05)
                    return True
                except queue.Full:
                    pass
            return False

        def reader():
            try:
                for k, off, ln in jobs:
                    while not free[k % 2].acquire(timeout=0.05):
                        if stop.is_set():
                            return
                    if fmap is not None:
                        crcs = _host.copy_crc32c_chunks(fmap[off:off + ln], slots[k % 2][:ln])
                    else:
                        crcs = read_slot(self.shm_src_path, slots[k % 2][:ln], off)
                    if not put((k, off, ln, crcs)):
                        return
            except Exception as e:  # noqa: BLE001
                put(e)
        th = threading.Thread(target=reader, daemon=True)
        tl = time.time()
        th.start()
        # the Adam moments are needed only by the first optimizer step: with the state on the device, restore the
        # master (and whatever shares its last piece) now, hand the moments to a background thread on a stream of
        # its own, and let the first step's forward / backward run meanwhile (the optimizer waits: _await_moments)
        defer = self.cuda and self.defer_moments and all(getattr(eng, s_).is_cuda for s_ in STATE)
        split = next((i for i, (_, off, _) in enumerate(jobs) if off >= 4 * n), len(jobs)) if defer else len(jobs)
        try:
            self._restore_pieces(jobs[:split], q, free, slots, dsts, m, check, waited)
        except BaseException:
            stop.set()
            th.join()
            raise
        self.restore_stats["loop_s"] = round(time.time() - tl, 2)

        def finish():
            self._restore_pieces(jobs[split:], q, free, slots, dsts, m, check, waited)
            if check and end % _host.CHUNK:  # the chunk straddling the fp32/bf16 boundary: verify it whole
                tail = torch.empty(min(_host.CHUNK, m["bytes"] - (end // _host.CHUNK) * _host.CHUNK),
                                   dtype=torch.uint8)
                c = read_slot(self.shm_src_path, tail, (end // _host.CHUNK) * _host.CHUNK)
                if c[0] != m["crc"][end // _host.CHUNK]:
                    raise CorruptCheckpoint("shm snapshot: checksum mismatch")
            self.restore_stats.update(wait_read_s=round(waited[0], 2), wait_h2d_s=round(waited[1], 2),
                                      pieces=len(jobs), piece_MiB=piece >> 20, GiB=round(end / 2 ** 30, 1))

        if split < len(jobs):
            self.restore_stats["deferred_GiB"] = round(sum(j[2] for j in jobs[split:]) / 2 ** 30, 1)
            td = time.time()
            stream = owned_stream(self.dev, "ckpt-restore", owner=self)

            def background():
                try:
                    with torch.cuda.stream(stream):
                        finish()
                        ev = torch.cuda.Event()
                        ev.record(stream)
                    self._moments_ev = ev
                except BaseException as e:  # noqa: BLE001 -- re-raised by _await_moments
                    self._moments_err = e
                finally:
                    stop.set()
                    th.join()
                    self.restore_stats["deferred_s"] = round(time.time() - td, 2)
            self._moments_err, self._moments_ev = None, None
            self._moments = threading.Thread(target=background, daemon=True, name="ckpt-restore-moments")
            self._moments.start()
            self.engine.pre_step_hooks.insert(0, self._await_moments)
        else:
            try:
                finish()
            finally:
                stop.set()
                th.join()
        # keep the mapping: unmapping ~90 GiB of populated page tables took ~3 s on the restore's critical
        # path, and the snapshot buffer the next save needs is this same file (_alloc_snapshot reuses it)
        self._restored_map = fmap
        eng.step_count = int(m["meta"]["global_steps"])
        self._loaded_meta = m["meta"]
        return m["meta"].get("client_state", {})

    def _await_moments(self, engine=None) -> None:
        """Join a deferred restore of the Adam moments (_load_shm): the host waits for the background thread to
        have queued its copies, the current stream for the copies. A checksum failure there ends the run loudly
        and marks the snapshot bad, so the relaunch falls back to an older candidate instead of this one."""
        th = self._moments
        if th is None:
            return
        th.join()
        self._moments = None
        if self._await_moments in self.engine.pre_step_hooks:
            self.engine.pre_step_hooks.remove(self._await_moments)
        # every rank deferred its moments (the same restore decision), so every rank reaches this point once, before
        # its first optimizer collective: agree on the outcome there. A checksum failure on ONE rank then fails every
        # rank together (the coordinated rollback load() promises), instead of leaving the healthy ranks blocked in
        # the gradient-statistics all-reduce until the process-group timeout
        ok = _Agree(self.engine).min(0.0 if self._moments_err is not None else 1.0)
        if self._moments_err is not None:
            try:
                with open(self.shm_src_meta + ".bad", "w") as f:
                    f.write(str(self._moments_err))
            except OSError:
                pass
            raise CorruptCheckpoint(f"shm snapshot: Adam moments failed to restore: {self._moments_err}")
        if ok < 1.0:
            raise CorruptCheckpoint("shm snapshot: Adam moments failed to restore on another rank")
        if self._moments_ev is not None:
            torch.cuda.current_stream(self.dev).wait_event(self._moments_ev)

    def _restore_pieces(self, jobs, q, free, slots, dsts, m, check, waited) -> None:
        """Main-thread half of the shm restore: verify each piece the reader copied and send it to the device."""
        for _ in jobs:
            tw = time.time()
            item = q.get()
            waited[0] += time.time() - tw
            if isinstance(item, Exception):
                raise item
            k, off, ln, crcs = item
            first, nfull = off // _host.CHUNK, ln // _host.CHUNK  # a partial last chunk is verified below
            if check and crcs[:nfull] != m["crc"][first:first + nfull]:
                raise CorruptCheckpoint("shm snapshot: checksum mismatch")
            src = slots[k % 2]
            self._touched = True
            for base, dst in dsts:
                lo, hi = max(off, base), min(off + ln, base + dst.numel())
                if lo < hi:
                    dst[lo - base:hi - base].copy_(src[lo - off:hi - off], non_blocking=True)
            if self.cuda:
                ev = torch.cuda.Event()
                ev.record()
                tw = time.time()
                ev.synchronize()
                waited[1] += time.time() - tw
            free[k % 2].release()

    def _load_tag(self, tag: str, verify: bool) -> Dict[str, Any]:
        d = os.path.join(self.save_dir, tag)
        if not os.path.exists(os.path.join(d, "COMPLETE")):
            raise CorruptCheckpoint("missing COMPLETE marker")
        # mmap: the module state dict (16-bit weights) in this file is not read by a restore
        meta = torch.load(os.path.join(d, MODEL0), weights_only=True, mmap=True)
        mans = {}
        for r in meta["writers"]:
            with open(os.path.join(d, f"manifest_r{r}.json")) as f:
                mans[r] = json.load(f)
            for fname in mans[r]["files"]:
                if not os.path.exists(os.path.join(d, fname)):
                    raise CorruptCheckpoint(f"{fname}: missing")
        src = _source_rank(self.engine)
        old = mans.get(src)
        same = old is not None and json.dumps(old["layout"], sort_keys=True) == json.dumps(
            dict(self.layout, rank=src), sort_keys=True)
        self._touched = True  # from here on the engine's state is being overwritten
        if same:
            info = old["files"][optim_file(src)]
            path = os.path.join(d, optim_file(src))
            for name in STATE:
                self._read_into(path, info[name], getattr(self.engine, name), verify)
        else:
            self._reshard_from(d, meta, mans, verify)
        self.engine.step_count = int(meta["global_steps"])
        self._loaded_meta = meta
        return meta.get("client_state", {})

    def _read_into(self, path: str, info: Dict[str, Any], dst: torch.Tensor, verify: bool) -> None:
        """Stream one slot into `dst` (device or host) through a pinned ring, verifying chunk CRCs."""
        n = dst.numel()
        if info["bytes"] != n * 4:
            raise CorruptCheckpoint(f"{os.path.basename(path)}: size mismatch")
        per = self.ring_elems
        ring = torch.empty(per, dtype=torch.float32, pin_memory=self.cuda)
        check = verify and info.get("algo") == _host.algo()
        for off in range(0, n, per):
            ln = min(per, n - off)
            crcs = read_slot(path, ring[:ln], info["offset"] + off * 4)
            first = off * 4 // _host.CHUNK
            if check and crcs != info["crc"][first:first + len(crcs)]:
                raise CorruptCheckpoint(f"{os.path.basename(path)}: checksum mismatch")
            dst[off:off + ln].copy_(ring[:ln], non_blocking=False)

    def _reshard_from(self, d: str, meta: Dict[str, Any], mans: Dict[int, Any], verify: bool) -> None:
        """Elastic restore: rebuild this rank's shards from a checkpoint written under another layout."""
        src = ShardSource(d, mans, verify)
        eng = self.engine
        ep_rank = self.layout["ep_rank"]
        for name in STATE:
            dst = getattr(eng, name)
            for g in eng.groups:
                full = src.assemble(g.name, g.kind, [(s.name, g.layout[s.name][0], list(s.shape), int(s.experts))
                                                     for s in g.specs], g.numel, name, ep_rank)
                r0 = (g.comm.rank if g.P > 1 else 0) * g.shard_numel
                dst.narrow(0, g.shard_off, g.shard_numel).copy_(torch.from_numpy(full[r0:r0 + g.shard_numel]))

    def discard_shm(self) -> None:
        """Drop the host-RAM snapshot tier (after a clean finish: nothing to resume)."""
        for p in (self.shm_meta, self.shm_path, self.shm_meta + ".bad"):
            try:
                os.unlink(p)
            except OSError:
                pass

    def close(self, discard_shm: bool = False) -> None:
        self._await_moments()
        self.wait()
        if self._before_optimizer_step in self.engine.pre_step_hooks:
            self.engine.pre_step_hooks.remove(self._before_optimizer_step)
        if self._prep is not None:  # background page-locking still running: stop it before unregistering
            self._reg_stop.set()
            self._prep.join()
            self._prep = None
        if self.cuda and self._reg:
            self._unregister_all()
        self._reg, self._reg_done, self._falloc_done, self._mapped_done = [], 0, 0, 0
        self._pinned_shm = False
        self._snap = None
        self._slots = []
        self._restored_map = None
        if discard_shm:
            self.discard_shm()


class ShardSource:
    """Old shard files of one checkpoint tag, memory-mapped; reassembles groups under any new layout.

    Dense groups are the concatenation of the old partition ranks' shards. Expert groups are rebuilt
    expert by expert: global expert j lived on old EP rank j // E_local_old (sharded over that EP
    position's expert-data-parallel ranks), so a new EP size just re-slices the global expert list."""

    def __init__(self, d: str, mans: Dict[int, Any], verify: bool = True):
        self.d, self.verify = d, verify
        self.mans = {int(r): m for r, m in mans.items()}
        self._maps: Dict[Tuple[int, str], np.ndarray] = {}
        self._verified: set = set()
        any_lay = next(iter(self.mans.values()))["layout"]
        self.W, self.stage, self.ep = any_lay["world"], any_lay["zero_stage"], any_lay["ep_size"]

    def _map(self, rank: int, state: str) -> np.ndarray:
        key = (rank, state)
        if key not in self._maps:
            info = self.mans[rank]["files"][optim_file(rank)][state]
            path = os.path.join(self.d, optim_file(rank))
            mm = np.memmap(path, dtype=np.float32, mode="r", offset=info["offset"], shape=(info["bytes"] // 4,))
            if self.verify and info.get("algo") == _host.algo() and key not in self._verified:
                ch = _host.CHUNK // 4
                got = [_host.crc32c_chunks(torch.from_numpy(np.array(mm[i:i + ch])))[0]
                       for i in range(0, mm.shape[0], ch)]
                if got != info["crc"][:len(got)]:
                    raise CorruptCheckpoint(f"{optim_file(rank)}:{state}: checksum mismatch")
                self._verified.add(key)
            self._maps[key] = mm
        return self._maps[key]

    def _group(self, rank: int, gname: str) -> Dict[str, Any]:
        for g in self.mans[rank]["layout"]["groups"]:
            if g["name"] == gname:
                return g
        raise KeyError(f"group {gname} not in rank {rank}'s checkpoint")

    def _old_flat(self, gname: str, state: str, ranks: List[int]) -> np.ndarray:
        """Full flat segment of group `gname` from the shards of `ranks` (in partition order)."""
        parts = []
        for r in ranks:
            g = self._group(r, gname)
            parts.append(self._map(r, state)[g["shard_off"]:g["shard_off"] + g["shard_numel"]])
        return np.concatenate(parts) if len(parts) > 1 else np.asarray(parts[0])

    def _holders(self, gname: str, kind: str, ep_rank: int) -> List[int]:
        """Old writer ranks holding group `gname` (for experts: of old EP position ep_rank), partition order."""
        if kind != "expert" or self.ep == 1:
            if self.stage == 0:
                return [0]
            rs = sorted(self.mans, key=lambda r: self._group(r, gname)["prank"])
            return rs[:1] if self._group(rs[0], gname)["P"] == 1 else rs  # replicated group: one copy
        rs = [r for r in self.mans if self.mans[r]["layout"]["ep_rank"] == ep_rank]
        return sorted(rs, key=lambda r: self._group(r, gname)["prank"])

    def assemble(self, gname: str, kind: str, params: List[Any], numel: int, state: str,
                 new_ep_rank: int = 0) -> np.ndarray:
        """The new full flat segment (numel elements) of group `gname` for new EP position `new_ep_rank`."""
        full = np.zeros(numel, dtype=np.float32)
        if kind != "expert":
            old = self._old_flat(gname, state, self._holders(gname, kind, 0))
            ref = self._group(self._holders(gname, kind, 0)[0], gname)
            old_off = {p[0]: p[1] for p in ref["params"]}
            for name, off, shape, _ in params:
                n = math.prod(shape)
                full[off:off + n] = old[old_off[name]:old_off[name] + n]
            return full
        cache: Dict[int, Tuple[np.ndarray, Dict[str, Any]]] = {}
        for name, off, shape, el_new in params:
            el_new = el_new or shape[0]
            per = math.prod(shape[1:])
            for k in range(el_new):
                j = new_ep_rank * el_new + k  # global expert id
                ref0 = self._group(next(iter(self.mans)), gname)
                el_old = next(p[3] or p[2][0] for p in ref0["params"] if p[0] == name)
                eo, lj = divmod(j, el_old)
                if eo not in cache:
                    holders = self._holders(gname, kind, eo)
                    if not holders:
                        raise CorruptCheckpoint(f"{gname}: no shard of old EP rank {eo}")
                    cache[eo] = (self._old_flat(gname, state, holders), self._group(holders[0], gname))
                old, og = cache[eo]
                ooff = next(p[1] for p in og["params"] if p[0] == name)
                full[off + k * per:off + (k + 1) * per] = old[ooff + lj * per:ooff + (lj + 1) * per]
        return full

    def consolidate(self, groups: List[Dict[str, Any]], state: str = "master") -> Dict[str, np.ndarray]:
        """Full named tensors (experts concatenated in global order) from the checkpoint alone."""
        out: Dict[str, np.ndarray] = {}
        for g in groups:
            if g.get("kind", "dense") != "expert" or self.ep == 1:
                holders = self._holders(g["name"], "dense", 0)
                flat = self._old_flat(g["name"], state, holders)
                for name, off, shape in (p[:3] for p in g["params"]):
                    out[f"{g.get('prefix', g['name'])}.{name}"] = np.array(flat[off:off + math.prod(shape)]).reshape(shape)
                continue
            per_ep = []
            for eo in range(self.ep):
                holders = self._holders(g["name"], "expert", eo)
                per_ep.append((self._old_flat(g["name"], state, holders), self._group(holders[0], g["name"])))
            for name, _, shape in (p[:3] for p in g["params"]):
                pieces = []
                for flat, og in per_ep:
                    ooff, oshape = next((p[1], p[2]) for p in og["params"] if p[0] == name)
                    pieces.append(np.array(flat[ooff:ooff + math.prod(oshape)]).reshape(oshape))
                out[f"{g.get('prefix', g['name'])}.{name}"] = np.concatenate(pieces)
        return out


def complete_tags(save_dir: str) -> List[str]:
    """Complete checkpoint tags sorted by step (oldest first)."""
    if not os.path.isdir(save_dir):
        return []
    out = []
    for t in os.listdir(save_dir):
        m = TAG_RE.match(t)
        if m and os.path.exists(os.path.join(save_dir, t, "COMPLETE")):
            out.append((int(m.group(1)), t))
    return [t for _, t in sorted(out)]


def export_consolidated(engine, path: str, dtype: torch.dtype = torch.bfloat16) -> Optional[str]:
    """``stage3_gather_16bit_weights_on_model_save``: gather full weights into one safetensors file (rank 0)."""
    from safetensors.torch import save_file

    params = engine.full_params()
    if engine.rank != 0:
        return None
    save_file({k: v.to(dtype).cpu().contiguous() for k, v in params.items()}, path)
    return path
