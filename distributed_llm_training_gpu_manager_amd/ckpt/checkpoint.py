"""Asynchronous sharded checkpoints with a DeepSpeed-style layout, integrity manifests and resharding.

The reference has no checkpoint code at all; its README claims
auto-resume (``README.md:14``) and its config asks DeepSpeed to gather 16-bit
weights on save (``ai_engine/deepspeed_launcher.py:74, :192``). This module is the
MI355X implementation (§2.5 N8):

Capture (training thread, no host sync)
    ``device`` mode: the rank's fp32 master / exp_avg / exp_avg_sq shards are copied
    D2D into a spare-HBM snapshot on a side stream (ZeRO-3 at W=8 is 12 B/param/8 --
    milliseconds at HBM bandwidth); ``host`` mode (not enough free HBM, e.g. W=1):
    D2H with ``non_blocking`` into pinned host memory. The next optimizer step
    waits for the capture event *on the GPU* (``stream.wait_event``), so training
    never blocks on the host.
Write-out (background thread, off the critical path)
    device mode streams the snapshot D2H through a 2-slot pinned ring; the C++ host
    runtime (``csrc/host/ckpt_io.cpp``) pwrites each piece with 8 threads and a CRC32C
    per 64 MiB chunk; files are fsync'ed; every rank writes ``manifest_r<r>.json``;
    rank 0 waits for all manifests, writes ``COMPLETE``, renames ``<tag>.tmp`` ->
    ``<tag>`` and atomically updates ``latest`` (no collectives from the writer thread).
Layout (names follow DeepSpeed; tensors in raw ``.bin`` files, metadata in ``.pt``
files loadable with ``torch.load(weights_only=True)``)::

    <save_dir>/latest                                    "global_step120"
    <save_dir>/global_step120/mp_rank_00_model_states.pt  engine/model metadata, group layout, client state
    <save_dir>/global_step120/zero_pp_rank_{r}_mp_rank_00_optim_states.pt   per-rank file index
    <save_dir>/global_step120/zero_pp_rank_{r}_mp_rank_00_optim_states.{master,exp_avg,exp_avg_sq}.bin
    <save_dir>/global_step120/manifest_r{r}.json  COMPLETE

Restore verifies sizes and CRCs while reading, falls back to the previous complete
tag when a file is missing or corrupt (rollback), and reshards when the world size
changed (elastic restart).
"""
from __future__ import annotations

import json
import os
import queue
import re
import shutil
import threading
import time
from typing import Any, Dict, List, Optional

import numpy as np
import torch

from .. import _host

STATE = ("master", "exp_avg", "exp_avg_sq")
TAG_RE = re.compile(r"^global_step(\d+)$")


class CorruptCheckpoint(RuntimeError):
    pass


def _tag(step: int) -> str:
    return f"global_step{step}"


def _optim_prefix(rank: int) -> str:
    return f"zero_pp_rank_{rank}_mp_rank_00_optim_states"


class AsyncCheckpointer:
    def __init__(self, engine, save_dir: str, mode: str = "auto", keep_last: int = 3,
                 ring_bytes: int = 1 << 30, manifest_timeout_s: float = 600.0):
        self.engine = engine
        self.save_dir = save_dir
        self.keep_last = keep_last
        self.rank = engine.rank if engine.P > 1 else 0
        self.P = engine.P
        self.is_writer_rank0 = engine.rank == 0
        # stage 0 (P == 1): every rank holds the full state; only rank 0 writes it
        self.active = self.P > 1 or engine.rank == 0
        self.n = engine.shard_total
        self.dev = engine.device
        self.cuda = self.dev.type == "cuda"
        self.ring_elems = max(_host.CHUNK // 4, (ring_bytes // 4) // (_host.CHUNK // 4) * (_host.CHUNK // 4))
        self.manifest_timeout_s = manifest_timeout_s
        self.mode = self._pick_mode(mode)
        self._snap: Optional[torch.Tensor] = None  # device: [3, n] fp32; host: pinned [3, n]
        self._ring: List[torch.Tensor] = []
        self._stream = torch.cuda.Stream(self.dev) if self.cuda else None
        self._capture_ev: Optional[torch.cuda.Event] = None
        self._pending = 0
        self._plock = threading.Lock()
        self._q: "queue.Queue" = queue.Queue()
        self._errors: List[str] = []
        self.history: List[Dict[str, Any]] = []
        self._thread = threading.Thread(target=self._writer, daemon=True, name="ckpt-writer")
        self._thread.start()
        engine.pre_step_hooks.append(self._before_optimizer_step)
        os.makedirs(save_dir, exist_ok=True)

    # ------------------------------------------------------------------ policy
    def _pick_mode(self, mode: str) -> str:
        if not self.cuda or getattr(self.engine, "offload", None) is not None:
            return "host"  # offloaded optimizer state already lives in host memory
        if mode != "auto":
            return mode
        free, _ = torch.cuda.mem_get_info(self.dev)
        need = 3 * self.n * 4
        return "device" if free > need + (24 << 30) else "host"

    def _before_optimizer_step(self, engine) -> None:
        # GPU-side ordering only: the next AdamW must not overwrite master/m/v before the capture read them
        if self._capture_ev is not None and self.cuda:
            torch.cuda.current_stream(self.dev).wait_event(self._capture_ev)

    # ------------------------------------------------------------------ save
    def save(self, step: int, client_state: Optional[Dict[str, Any]] = None, blocking: bool = False) -> str:
        t0 = time.time()
        if not self.active:
            return _tag(step)
        if self.busy:  # previous write-out still streaming from the snapshot buffer
            self.wait()
        tag = _tag(step)
        tmp = os.path.join(self.save_dir, tag + ".tmp")
        os.makedirs(tmp, exist_ok=True)
        eng = self.engine
        srcs = [eng.master, eng.exp_avg, eng.exp_avg_sq]
        if self._snap is None:
            if self.mode == "device":
                self._snap = torch.empty((3, self.n), dtype=torch.float32, device=self.dev)
                self._ring = [torch.empty(self.ring_elems, dtype=torch.float32, pin_memory=True) for _ in range(2)]
            else:
                self._snap = torch.empty((3, self.n), dtype=torch.float32, pin_memory=self.cuda)
        if self.cuda:
            cur = torch.cuda.current_stream(self.dev)
            self._stream.wait_stream(cur)
            with torch.cuda.stream(self._stream):
                for i, s in enumerate(srcs):
                    self._snap[i].copy_(s, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self._stream)
            self._capture_ev = ev
        else:
            for i, s in enumerate(srcs):
                self._snap[i].copy_(s)
            ev = None
        meta = self._meta(step, client_state or {})
        with self._plock:
            self._pending += 1
        self._q.put((tag, tmp, step, ev, meta, t0))
        if blocking:
            self.wait()
        return tag

    def _meta(self, step: int, client_state: Dict[str, Any]) -> Dict[str, Any]:
        eng = self.engine
        ecfg = {k: (str(v) if isinstance(v, torch.dtype) else list(v) if isinstance(v, tuple) else v)
                for k, v in vars(eng.cfg).items()}
        groups = [{"name": g.name, "numel": g.numel, "shard_numel": g.shard_numel, "shard_off": g.shard_off,
                   "params": [[s.name, g.layout[s.name][0], list(s.shape)] for s in g.specs]} for g in eng.groups]
        return {"ds_version": "dlgm-mi355x-0.1", "global_steps": step, "dp_world_size": eng.W,
                "partition_count": self.P, "zero_stage": eng.stage, "model_config": eng.mcfg.to_dict(),
                "engine_config": ecfg, "groups": groups, "shard_total": self.n, "client_state": client_state,
                "lr_scheduler": {"step": step}, "param_shapes": {g["name"]: {p[0]: p[2] for p in g["params"]}
                                                                  for g in groups}}

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

    def _writer(self) -> None:
        while True:
            tag, tmp, step, ev, meta, t0 = self._q.get()
            try:
                self._write_one(tag, tmp, step, ev, meta, t0)
            except Exception as e:  # noqa: BLE001
                self._errors.append(f"{tag}: {e}")
            finally:
                with self._plock:
                    self._pending -= 1

    def _write_one(self, tag: str, tmp: str, step: int, ev, meta: Dict[str, Any], t0: float) -> None:
        if ev is not None:
            while not ev.query():
                time.sleep(0.0005)
        t_cap = time.time()
        prefix = _optim_prefix(self.rank)
        files = {}
        for i, name in enumerate(STATE):
            fname = f"{prefix}.{name}.bin"
            path = os.path.join(tmp, fname)
            nbytes = self.n * 4
            w = _host.StreamWriter(path, nbytes)
            if self.mode == "device":
                for k, off in enumerate(range(0, self.n, self.ring_elems)):
                    ln = min(self.ring_elems, self.n - off)
                    slot = self._ring[k % 2]
                    with torch.cuda.stream(self._stream):
                        slot[:ln].copy_(self._snap[i, off:off + ln], non_blocking=True)
                        e2 = torch.cuda.Event()
                        e2.record(self._stream)
                    e2.synchronize()  # this background thread only
                    w.write(slot[:ln], off * 4)
            else:
                w.write(self._snap[i], 0)
            crcs = w.close(fsync=True)
            files[fname] = {"bytes": nbytes, "chunk": _host.CHUNK, "crc": crcs, "algo": _host.algo(), "tensor": name}
        torch.save({"rank": self.rank, "partition_count": self.P, "shard_numel": self.n, "files": sorted(files),
                    "optimizer": {"type": "AdamW", "step": step}}, os.path.join(tmp, prefix + ".pt"))
        if self.is_writer_rank0:
            torch.save(meta, os.path.join(tmp, "mp_rank_00_model_states.pt"))
        man = {"rank": self.rank, "partition_count": self.P, "step": step, "files": files}
        mtmp = os.path.join(tmp, f".manifest_r{self.rank}.json")
        with open(mtmp, "w") as f:
            json.dump(man, f)
        os.replace(mtmp, os.path.join(tmp, f"manifest_r{self.rank}.json"))
        rec = {"tag": tag, "step": step, "capture_s": t_cap - t0, "write_s": time.time() - t_cap,
               "bytes": 3 * self.n * 4, "mode": self.mode}
        if self.is_writer_rank0:
            deadline = time.time() + self.manifest_timeout_s
            while time.time() < deadline:
                if all(os.path.exists(os.path.join(tmp, f"manifest_r{r}.json")) for r in range(self.P)):
                    break
                time.sleep(0.05)
            else:
                raise TimeoutError(f"{tag}: not all ranks wrote their manifests")
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
            rec["published_s"] = time.time() - t0
        self.history.append(rec)

    def _prune(self) -> None:
        tags = complete_tags(self.save_dir)
        for t in tags[:-self.keep_last] if self.keep_last > 0 else []:
            shutil.rmtree(os.path.join(self.save_dir, t), ignore_errors=True)

    # ------------------------------------------------------------------ restore
    def load(self, tag: str = "auto", verify: bool = True) -> Optional[Dict[str, Any]]:
        """Restore engine state; returns the client state (None when no checkpoint exists).

        ``tag="auto"``: newest complete tag whose files verify -- a corrupt or partial
        newest tag is skipped (rolled back) with a warning recorded in ``self.rollbacks``.
        """
        self.rollbacks: List[str] = []
        cands = [tag] if tag not in ("auto", "latest") else list(reversed(complete_tags(self.save_dir)))
        for t in cands:
            try:
                return self._load_tag(t, verify)
            except (CorruptCheckpoint, FileNotFoundError, OSError, KeyError) as e:
                self.rollbacks.append(f"{t}: {e}")
                if tag not in ("auto", "latest"):
                    raise
        return None

    def _load_tag(self, tag: str, verify: bool) -> Dict[str, Any]:
        d = os.path.join(self.save_dir, tag)
        if not os.path.exists(os.path.join(d, "COMPLETE")):
            raise CorruptCheckpoint("missing COMPLETE marker")
        meta = torch.load(os.path.join(d, "mp_rank_00_model_states.pt"), weights_only=True)
        eng = self.engine
        oldP = meta["partition_count"]
        mans = {}
        for r in range(oldP):
            with open(os.path.join(d, f"manifest_r{r}.json")) as f:
                mans[r] = json.load(f)
            for fname, info in mans[r]["files"].items():
                p = os.path.join(d, fname)
                if os.path.getsize(p) != info["bytes"]:
                    raise CorruptCheckpoint(f"{fname}: size mismatch")
        if oldP == self.P and [g["numel"] for g in meta["groups"]] == [g.numel for g in eng.groups]:
            buf = torch.empty(self.n, dtype=torch.float32, pin_memory=self.cuda)
            prefix = _optim_prefix(self.rank)
            for name in STATE:
                fname = f"{prefix}.{name}.bin"
                crcs = _host.read_tensor(os.path.join(d, fname), buf)
                info = mans[self.rank]["files"][fname]
                if verify and info["algo"] == _host.algo() and crcs != info["crc"]:
                    raise CorruptCheckpoint(f"{fname}: checksum mismatch")
                getattr(eng, name).copy_(buf, non_blocking=False)
        else:
            self._reshard_from(d, meta, mans, verify)
        eng.step_count = int(meta["global_steps"])
        eng.sync_params_from_master()
        return meta.get("client_state", {})

    def _reshard_from(self, d: str, meta: Dict[str, Any], mans: Dict[int, Any], verify: bool) -> None:
        """Elastic restore: rebuild this rank's shards from the old world's shard files."""
        eng = self.engine
        oldP = meta["partition_count"]
        old_groups = {g["name"]: g for g in meta["groups"]}
        for name in STATE:
            maps = [np.memmap(os.path.join(d, f"{_optim_prefix(r)}.{name}.bin"), dtype=np.float32, mode="r")
                    for r in range(oldP)]
            dst = getattr(eng, name)
            for g in eng.groups:
                og = old_groups[g.name]
                full = np.zeros(g.numel, dtype=np.float32)
                n = min(og["numel"], g.numel)
                pos = 0
                for r in range(oldP):
                    seg = maps[r][og["shard_off"]:og["shard_off"] + og["shard_numel"]]
                    take = max(0, min(len(seg), n - pos))
                    full[pos:pos + take] = seg[:take]
                    pos += len(seg)
                r0 = (eng.rank if self.P > 1 else 0) * g.shard_numel
                dst.narrow(0, g.shard_off, g.shard_numel).copy_(torch.from_numpy(full[r0:r0 + g.shard_numel]))
            del maps

    def close(self) -> None:
        self.wait()
        if self._before_optimizer_step in self.engine.pre_step_hooks:
            self.engine.pre_step_hooks.remove(self._before_optimizer_step)


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
