"""Training loop: the script the launcher runs on every rank (``python -m distributed_llm_training_gpu_manager_amd.train``).

Contract kept from DeepSpeed scripts: it takes ``--deepspeed_config=<json>`` (the
file written by the launcher) and reads ``RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*`` from
the environment (``torch.distributed.run``). Everything the reference delegates to a
user script is here: synthetic data, the ZeRO engine, in-process
loss monitoring, the NaN trap, async checkpoints, auto-resume and spot preemption.

Exit codes (read by the supervisor): 0 done, 3 NaN/Inf halt, 4 preempted (emergency
checkpoint written), 5 transport failure (an xGMI mesh wait timed out or an EP dispatch overflowed:
the supervisor resumes from the newest verified checkpoint). Rank 0 publishes per-step progress to
``DLGM_STATUS_FILE``; every rank writes its heartbeat to ``DLGM_HEARTBEAT_DIR`` (hang detection).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import queue
import signal
import sys
import threading
import time
import urllib.request
from typing import Any, Dict, List, Optional, Tuple

import torch

from ..ckpt.checkpoint import AsyncCheckpointer, export_consolidated
from ..health.loss_monitor import json_safe, LossSpikeMonitor, MonitorConfig, TrainingMetrics
from ..health.nan_trap import NanTrap
from ..launcher.supervisor import (EXIT_EP_OVERFLOW, EXIT_NAN_HALT, EXIT_PREEMPTED, EXIT_TRANSPORT, write_heartbeat,
                                   write_status)
from ..models import get_config
from ..parallel.comm import Comm, init_distributed
from ..parallel.zero import EngineConfig, ZeroEngine
from ..utils.profiling import trace_window
from .dsconfig import engine_config_from_ds



class HeartbeatTicker:
    """Heartbeats from a side thread while this rank blocks outside the step loop -- the final checkpoint write-out,
    export_consolidated, a blocking emergency save, a save waiting for the previous write-out: the
    supervisor's hang bound is sized to the step time, and those phases can take minutes on a large model or a slow
    disk. The beats carry ``phase`` (BLOCKING_PHASES: the supervisor applies its start-up bound) and
    ``blocked_since`` (a block longer than BLOCK_LIMIT_MULT bounds is still a hang)."""

    def __init__(self, rank: int, step: int, phase: str, interval_s: float = 5.0):
        self.rank, self.step, self.phase, self.interval_s = rank, step, phase, interval_s
        self._stop = threading.Event()
        self._t: Optional[threading.Thread] = None

    def _beat(self, since: float) -> None:
        write_heartbeat(self.rank, self.step, phase=self.phase, blocked_since=since)

    def __enter__(self):
        since = time.time()
        self._beat(since)

        def run():
            while not self._stop.wait(self.interval_s):
                self._beat(since)
        self._t = threading.Thread(target=run, daemon=True, name=f"heartbeat-{self.phase}")
        self._t.start()
        return self

    def __exit__(self, *exc):
        self._stop.set()
        if self._t is not None:
            self._t.join()
        return False

class SyntheticData:
    """Deterministic random token batches: (seed, rank, step, micro) -> the same tokens after a restart."""

    def __init__(self, vocab: int, mbs: int, seq: int, ga: int, seed: int, rank: int, device: torch.device,
                 sp_rank: int = 0, sp_size: int = 1):
        """`rank` is the data-parallel rank; under sequence parallelism every rank of an SP group draws
        the same full sequences and keeps its own contiguous chunk of seq / sp_size tokens."""
        self.vocab, self.mbs, self.seq, self.ga = vocab, mbs, seq, ga
        self.seed, self.rank, self.device = seed, rank, device
        self.sp_rank, self.sp_size = sp_rank, sp_size
        self.gen = torch.Generator(device=device)

    def batches(self, step: int) -> List[Tuple[torch.Tensor, torch.Tensor]]:
        out = []
        n = self.seq // self.sp_size
        sl = slice(self.sp_rank * n, (self.sp_rank + 1) * n)
        for mi in range(self.ga):
            self.gen.manual_seed(((self.seed * 1_000_003 + self.rank) * 1_000_003 + step) * 131 + mi)
            toks = torch.randint(0, self.vocab, (self.mbs, self.seq + 1), device=self.device, generator=self.gen)
            out.append((toks[:, :-1][:, sl].contiguous(), toks[:, 1:][:, sl].contiguous()))
        return out


class MetricsPusher:
    """Best-effort, non-blocking POST of TrainingMetrics to the control plane's /monitoring/ingest.

    One sender thread drains a queue, so batches arrive in step order (the monitor's rules and the
    Prometheus step gauge depend on it) and the training loop never waits on HTTP."""

    def __init__(self, url: Optional[str], job_id: str):
        self.url, self.job_id = url, job_id
        self._q: "queue.Queue[Optional[Dict[str, Any]]]" = queue.Queue()
        self._thread: Optional[threading.Thread] = None
        if url:
            self._thread = threading.Thread(target=self._loop, daemon=True, name="metrics-push")
            self._thread.start()

    def push(self, m: Dict[str, Any]) -> None:
        if self.url:
            self._q.put(m)

    def _loop(self) -> None:
        while True:
            m = self._q.get()
            if m is None:
                return
            batch = [m]
            while True:  # coalesce whatever queued up while the last POST was in flight
                try:
                    nxt = self._q.get_nowait()
                except queue.Empty:
                    break
                if nxt is None:
                    self._send(batch)
                    return
                batch.append(nxt)
            self._send(batch)

    def _send(self, batch) -> None:
        body = json.dumps({"job_id": self.job_id, "metrics": batch}).encode()
        req = urllib.request.Request(self.url.rstrip("/") + "/api/v1/monitoring/ingest", data=body,
                                     headers={"content-type": "application/json"}, method="POST")
        try:
            urllib.request.urlopen(req, timeout=2).read()
        except Exception:  # noqa: BLE001
            pass

    def close(self, timeout_s: float = 5.0) -> None:
        if self._thread is not None:
            self._q.put(None)
            self._thread.join(timeout_s)


def _process_start() -> float:
    try:
        import psutil
        return float(psutil.Process().create_time())
    except Exception:  # noqa: BLE001
        return _T_IMPORTED


_T_IMPORTED = time.time()  # this module (and torch) imported


class Trainer:
    def __init__(self, args: argparse.Namespace):
        self.args = args
        # restart timeline (MTTR breakdown): process start -> imports -> process group -> engine -> restore ->
        # first completed step; printed once after the first step
        self.timeline: Dict[str, float] = {"process_start": _process_start(), "imported": _T_IMPORTED}
        self.env = init_distributed(args.device)
        self.timeline["dist_init"] = time.time()
        self.mem_notes: Dict[str, float] = {}
        if self.env.device.type == "cuda":  # HBM still held by a killed predecessor shows up here
            self.mem_notes["gpu_free_at_start_GiB"] = round(torch.cuda.mem_get_info(self.env.device)[0] / 2 ** 30, 1)
        self.comm = Comm()
        self.shadow = int(getattr(args, "shadow_world", 0) or 0)
        if self.shadow > 1:
            # rank `shadow_rank` of a world-`shadow_world` job alone on this GPU (parallel/comm.py ShadowComm, async
            # RCCL-ordered streams): its true-size shards, gathers, snapshot and restore -- the config-4 drill at
            # 70B rank scale on one MI355X
            from ..parallel.comm import ShadowComm
            assert self.env.world == 1, "--shadow-world runs one process"
            self.comm = ShadowComm(self.shadow, int(args.shadow_rank), async_mode=True)
        over = {"max_seq_len": max(args.seq_len, 1)} if args.seq_len else {}
        if getattr(args, "n_layers", 0):
            over["n_layers"] = args.n_layers  # drills on a box: the named architecture, fewer blocks
        self.mcfg = get_config(args.model, **over)
        if args.deepspeed_config:
            self.ecfg, self.notes = engine_config_from_ds(args.deepspeed_config, args.seq_len, seed=args.seed,
                                                          model_cfg=self.mcfg, world=self.env.world)
            with open(args.deepspeed_config) as f:
                self._ds_elastic = bool(json.load(f).get("elasticity", {}).get("enabled", False))
        else:
            self.ecfg, self.notes = EngineConfig(zero_stage=args.zero_stage, micro_batch_size=args.micro_batch,
                                                 seq_len=args.seq_len, grad_accum=args.grad_accum, lr=args.lr,
                                                 seed=args.seed, fp16=getattr(args, "fp16", False)), []
        if getattr(args, "auto_micro_batch", False) and not args.deepspeed_config:
            from .dsconfig import _auto_micro_batch
            _auto_micro_batch(self.ecfg, {"train_micro_batch_size_per_gpu": args.micro_batch}, self.mcfg,
                              self.env.world, self.notes)
        if args.lr_scale != 1.0:
            self.ecfg.lr *= args.lr_scale
        if getattr(args, "expert_parallel", 0):
            self.ecfg.expert_parallel_size = args.expert_parallel
        if getattr(args, "sequence_parallel", 0):
            # --seq-len is the FULL sequence; each rank of the SP group holds one contiguous chunk
            assert args.seq_len % args.sequence_parallel == 0, "--seq-len must divide by --sequence-parallel"
            self.ecfg.sequence_parallel_size = args.sequence_parallel
        self.sp = max(1, self.ecfg.sequence_parallel_size)
        self.ecfg.seq_len = args.seq_len // self.sp
        if getattr(args, "wall_clock_breakdown", False):
            self.ecfg.wall_clock_breakdown = True
        if getattr(args, "hip_graphs", False):
            self.ecfg.hip_graphs = True
        if getattr(args, "xgmi_mesh", None):
            self.ecfg.xgmi_mesh = args.xgmi_mesh
        if getattr(args, "activation_checkpointing", False):
            self.ecfg.activation_checkpointing = True  # the reference's 70b preset sets it (deepspeed_launcher.py:402)
        if args.halt_on_nan and not self.ecfg.fp16:
            self.ecfg.nan_latch = True  # the host runs one step ahead of the NaN decision (see NanTrap)
        self.global_batch = self._elastic_batch(args)
        save_dir = args.save_dir or os.environ.get("DLGM_SAVE_DIR")
        self.engine = ZeroEngine(self.mcfg, self.ecfg, self.env.device, self.comm)
        self.timeline["engine"] = time.time()
        if self.env.device.type == "cuda":
            self.mem_notes["gpu_free_after_engine_GiB"] = round(torch.cuda.mem_get_info(self.env.device)[0] / 2 ** 30, 1)

        self.monitor = LossSpikeMonitor(MonitorConfig())
        self.trap = NanTrap(self.env.device, self.monitor, width=6)
        shm = {"auto": "auto", "on": True, "off": False}[args.ckpt_shm]
        self.ckpt = AsyncCheckpointer(self.engine, save_dir, mode=args.ckpt_mode, keep_last=args.keep_last, shm=shm,
                                      disk=bool(args.ckpt_disk)) if save_dir else None
        drank = self.comm.rank if self.shadow > 1 else self.env.rank
        self.data = SyntheticData(self.mcfg.vocab_size, self.ecfg.micro_batch_size, args.seq_len,
                                  self.ecfg.grad_accum, args.seed, drank // self.sp, self.env.device,
                                  sp_rank=drank % self.sp, sp_size=self.sp)
        self.pusher = MetricsPusher(args.metrics_url if self.env.rank == 0 else None,
                                    os.environ.get("DLGM_JOB_ID", args.job_id))
        self.telemetry = None
        if self.env.device.type == "cuda" and args.telemetry_interval > 0:
            # amdsmi polling of this rank's GPU inside the job (BASELINE config 2: thermals / HBM)
            from ..health.telemetry import TelemetrySampler
            self.telemetry = TelemetrySampler(self.env.device, interval_s=args.telemetry_interval).start()
        self.preempt = False
        signal.signal(signal.SIGUSR1, self._on_preempt)
        signal.signal(signal.SIGTERM, self._on_preempt)
        self.log: List[Dict[str, Any]] = []
        self.read_behind = 0  # step reports read while the next step was already queued

    def _on_preempt(self, signum, frame) -> None:
        self.preempt = True

    def _elastic_batch(self, args) -> int:
        """Elastic training (DeepSpeed ``elasticity`` block, reference ``deepspeed_launcher.py:78, 226-238``):
        the global batch of the first launch is kept across restarts at other world sizes by rescaling the
        gradient accumulation; the number travels in the checkpoint's client state."""
        e = self.ecfg
        dp = max(1, self.env.world // max(1, e.sequence_parallel_size))
        gb = e.micro_batch_size * e.grad_accum * dp
        elastic = getattr(args, "elastic", False) or bool(getattr(self, "_ds_elastic", False))
        save_dir = args.save_dir or os.environ.get("DLGM_SAVE_DIR")
        if not elastic or not save_dir or args.resume in ("none", ""):
            return gb
        from ..ckpt.checkpoint import MODEL0, complete_tags
        tags = complete_tags(save_dir)
        if tags:
            meta = torch.load(os.path.join(save_dir, tags[-1], MODEL0), weights_only=True)
            gb = int(meta.get("client_state", {}).get("global_batch", gb))
        ga = max(1, round(gb / (e.micro_batch_size * dp)))
        if ga != e.grad_accum:
            self.notes.append(f"elastic: world {self.env.world} -> grad_accum {e.grad_accum} -> {ga} "
                              f"(global batch {gb}{'' if ga * e.micro_batch_size * dp == gb else ' not divisible: now ' + str(ga * e.micro_batch_size * dp)})")
            e.grad_accum = ga
        return ga * e.micro_batch_size * dp

    def _notice_due(self, step: int, first_attempt: bool) -> bool:
        """Spot drill: deliver the preemption notice after step --preempt-at-step; with --preempt-when-ready, after
        the first step from there on at which the snapshot buffer is prepared (a notice that lands on a warm job,
        the usual case hours into a run, rather than seconds after its start)."""
        a = self.args
        if a.preempt_at_step < 0 or self._notice_sent or not first_attempt or a.preempt_rank not in (-1, self.env.rank):
            return False
        if not a.preempt_when_ready:
            return step == a.preempt_at_step
        return step >= a.preempt_at_step and (self.ckpt is None or self.ckpt.prepared)

    def _say(self, msg: str) -> None:
        if self.env.rank == 0:
            print(f"[train] {msg}", flush=True)

    def _report(self, step: int, issued: Dict[str, Any]) -> Dict[str, Any]:
        """Read step `step`'s report (stats + loss) from the pinned ring: called for step t-1 right after
        step t is queued, so the wait overlaps step t on the GPU. The values are all-reduced, so every
        rank takes the same halt / preemption decision at the same loop iteration."""
        v = self.trap.get(step)
        if v is None:
            v = [float(x) for x in self._report_vector(issued["m"]).tolist()]
        ss, bad, flag, loss, gnorm, transport = v[0], v[1], v[2], v[3], v[4], v[5]
        now = time.time()
        dt = now - self._t_last
        self._t_last = now
        rec = {"step": step, "loss": loss, "grad_norm": gnorm,
               "lr": issued["m"]["lr"], "step_s": dt, "tokens_per_sec": self._tokens_step / max(dt, 1e-9),
               "nonfinite": bad, "preempt": flag > 0, "transport": int(transport)}
        self.log.append(rec)
        self._reports += 1
        if self._reports > 1:  # (the first report's time includes the warm-up)
            self._last_step_s = dt
        self._last_reported = step
        a = self.args
        if self.env.rank == 0:
            write_status(step, loss=loss, nonfinite=bad)
            if "first_step" not in self.timeline:
                self.timeline["first_step"] = now
                t = self.timeline
                keys = ["process_start", "imported", "dist_init", "engine", "restored", "first_step"]
                self._say("startup: " + json.dumps({f"{b}_s": round(t[b] - t[a_], 2) for a_, b in zip(keys, keys[1:])}
                                                    | {"total_s": round(now - t["process_start"], 2)}
                                                    | self.mem_notes))
            hbm = self.telemetry.aggs["hbm_used_gib"].max if self.telemetry is not None else None
            alerts = self.monitor.ingest(TrainingMetrics(step=step, loss=loss, learning_rate=rec["lr"],
                                                         gradient_norm=rec["grad_norm"],
                                                         tokens_per_sec=rec["tokens_per_sec"],
                                                         gpu_memory_used_mib=int(hbm * 1024) if hbm else 0))
            self.pusher.push({"step": step, "loss": loss if math.isfinite(loss) else 1e30,
                              "learning_rate": rec["lr"], "gradient_norm": rec["grad_norm"]
                              if math.isfinite(rec["grad_norm"]) else 1e30})
            if step % a.log_interval == 0 and self.engine.timers.enabled:
                rec["wall_clock_breakdown_ms"] = {k: v["total_ms"] for k, v in self.engine.timers.summary().items()}
            if step % a.log_interval == 0 or alerts:
                self._say(json.dumps(json_safe(rec)) + ("" if not alerts else f" alerts={[x.alert_type for x in alerts]}"))
        return rec

    def _report_vector(self, m: Dict[str, Any]) -> torch.Tensor:
        """[sum g^2, non-finite, flags, loss, unscaled grad norm, transport word] of the step just queued (device)."""
        return torch.cat([self.engine.stats, m["loss"].reshape(1).float(), m["grad_norm"].reshape(1).float(),
                          self.engine.transport_word()])

    def _decide(self, rec: Dict[str, Any], last_issued: int) -> Optional[int]:
        """Exit code to stop with after step rec['step'] (None: go on). `last_issued` has been queued too;
        with the NaN latch its update is skipped on the device, so a NaN halt leaves the pre-NaN state."""
        a = self.args
        if rec.get("transport"):
            # the mesh's sticky words (1: a device-side wait timed out, 2: an EP dispatch overflowed an explicit
            # capacity): the step trained on data nobody can vouch for -- stop without saving it; the supervisor
            # resumes from the newest verified checkpoint
            self._say(f"xGMI mesh transport failure at step {rec['step']} (word {rec['transport']}); halting")
            try:
                self.engine.check_transport()
            except RuntimeError as e:
                self._say(str(e))
            word = int(rec["transport"])
            # word 1: a wait timed out (resumable); word 2 alone: an explicit EP capacity overflowed (not resumable)
            return EXIT_EP_OVERFLOW if (word & 2) and not (word & 1) else EXIT_TRANSPORT
        if rec["nonfinite"] > 0 and a.halt_on_nan:
            self._say(f"NaN/Inf gradients at step {rec['step']} ({int(rec['nonfinite'])} elements): update skipped "
                      f"on device; halting")
            return EXIT_NAN_HALT
        if rec["preempt"]:
            t0 = time.time()
            if self.ckpt is not None:
                self.ckpt.save(last_issued, client_state={"step": last_issued, "preempted": True,
                                                                 "global_batch": self.global_batch}, blocking=True)
            self._say(f"preemption: emergency checkpoint at step {last_issued} in {time.time() - t0:.2f}s; exiting")
            if self.ckpt is not None and self.ckpt.history:
                self._say("emergency checkpoint record: " + json.dumps(json_safe(self.ckpt.history[-1])))
            return EXIT_PREEMPTED
        return None

    def run(self) -> int:
        a = self.args
        start = 0
        if self.ckpt is not None and a.resume not in ("none", ""):
            t0 = time.time()
            cs = self.ckpt.load("auto" if a.resume in ("auto", "latest") else a.resume)
            if cs is not None:
                start = int(cs.get("step", self.engine.step_count))
                self._say(f"resumed from step {start} in {time.time() - t0:.2f}s via {self.ckpt.restored_from} "
                          f"(rollbacks: {getattr(self.ckpt, 'rollbacks', [])}; "
                          f"restore {json.dumps(getattr(self.ckpt, 'restore_stats', {}))})")
                self.monitor.reset()
        self.timeline["restored"] = time.time()
        # snapshot buffer allocated / page-locked in the background while the first steps run. Page-locking
        # ~100 GB contends with kernel launches for seconds, so after a restore it starts once the first step
        # has completed: recovery (MTTR) is not held up by a buffer the next save needs.
        self._prep_after_first = self.ckpt is not None and start > 0
        if self.ckpt is not None and not self._prep_after_first:
            self.ckpt.prepare_async()
        for n in self.notes:
            self._say(f"note: {n}")
        self._tokens_step = self.ecfg.micro_batch_size * self.ecfg.seq_len * self.ecfg.grad_accum * self.env.world
        self._t_last = time.time()
        self._reports, self._last_step_s, self._last_reported = 0, None, start
        self._step_timing = int(os.environ.get("DLGM_STEP_TIMING", "0") or 0)
        write_heartbeat(self.env.rank, start, phase="ready")  # restored / initialised: the first step is next
        self._hb_tick = float(os.environ.get("DLGM_HEARTBEAT_TICK_S", "5"))
        self.engine.sync_flags = self.env.world > 1
        first_attempt = os.environ.get("DLGM_RESTART", "0") == "0"
        self._notice_sent = False
        rc = 0
        prev: Optional[Tuple[int, Dict[str, Any]]] = None
        last = start
        for step in range(start + 1, a.steps + 1):
            # every rank's own heartbeat, before it issues the step: a rank that stops (SIGSTOP, a hang in its own
            # code) goes stale first, the ranks waiting for it in their next collective one step later
            write_heartbeat(self.env.rank, self._last_reported, issuing=step, step_s=self._last_step_s)
            if a.inject_nan_step == step and first_attempt and a.inject_nan_rank in (-1, self.env.rank):
                # one faulty rank among healthy ones (--inject-nan-rank): the non-finite count rides the all-reduced
                # gradient statistics, so every rank skips the update and halts at the same step
                self.engine.fault_inject_nan = True
            self.engine.host_flag = 1.0 if self.preempt else 0.0
            prof = getattr(a, "profile_steps", 0) and step - start == 2  # trace window after one warm step
            t_iss = time.time()
            with trace_window(a.profile_dir if prof else None, self.env.rank):
                m = self.engine.train_step(self.data.batches(step))
                for _ in range(a.profile_steps - 1 if prof else 0):  # extra traced steps reuse this step's data
                    self.engine.train_step(self.data.batches(step))
            if self._step_timing and step - start <= self._step_timing and self.env.device.type == "cuda":
                # diagnostic (DLGM_STEP_TIMING=N: the first N steps of this attempt): host issue time vs device time
                t_q = time.time()
                torch.cuda.synchronize(self.env.device)
                self._say(f"step-timing: step {step} issue {t_q - t_iss:.3f}s device-done {time.time() - t_iss:.3f}s")
            # [sum g^2, non-finite, flags, loss, unscaled grad norm, transport]: read one step late from the pinned
            # ring (no sync in the loop); the fp16 loss scale stays on the device
            self.trap.record(step, self._report_vector(m))
            issued = {"m": m}
            last = step
            # step t-1's outcome, read while step t runs on the device
            if prev is not None:
                self.read_behind += 1  # read with a later step already queued behind it
                stop = self._decide(self._report(*prev), step)
                prev = None
                if self._prep_after_first:
                    self._prep_after_first = False
                    self.ckpt.prepare_async()
                if stop is not None:
                    rc = stop
                    break
            save_due = self.ckpt is not None and a.save_interval > 0 and step % a.save_interval == 0
            # the first step of a resumed attempt is read at once: recovery (the supervisor's MTTR) is confirmed when
            # that step is done, not one step later
            confirm = start > 0 and step == start + 1
            if save_due or confirm:  # never persist a step before knowing it is clean
                rec = self._report(step, issued)
                stop = self._decide(rec, step)
                if stop is not None:
                    rc = stop
                    break
                if self._prep_after_first:
                    self._prep_after_first = False
                    self.ckpt.prepare_async()
                if save_due:  # may wait for the previous write-out
                    with HeartbeatTicker(self.env.rank, step, "saving", self._hb_tick):
                        self.ckpt.save(step, client_state={"step": step, "global_batch": self.global_batch})
            else:
                prev = (step, issued)
            if a.kill_at_step == step and first_attempt and self.env.rank == a.kill_rank:
                if self.ckpt is not None:  # the drill kills after the last interval checkpoint is published
                    self.ckpt.wait()
                    last_saved = step - step % a.save_interval if a.save_interval > 0 else 0
                    if last_saved > 0:
                        self.ckpt.wait_published(last_saved)
                os.kill(os.getpid(), signal.SIGKILL)
            if a.stop_at_step == step and first_attempt and self.env.rank == a.stop_rank:
                os.kill(os.getpid(), signal.SIGSTOP)  # hang drill: this rank freezes (only SIGKILL / SIGCONT move it)
            if self._notice_due(step, first_attempt):
                # a notice on one rank only (--preempt-rank): its flag rides the next step's all-reduced statistics
                self._notice_sent = True
                os.kill(os.getpid(), signal.SIGUSR1)
            if self.preempt and self.env.world == 1:
                # one rank needs no agreement: checkpoint the step just queued, now (W > 1 ranks agree through
                # the flag slot of the next step's all-reduced stats)
                if prev is not None:  # prev is this step (not read yet): never persist a NaN step
                    rec = self._report(*prev)
                    prev = None
                    if rec["nonfinite"] > 0 and a.halt_on_nan:
                        rc = self._decide(rec, step)
                        break
                t0 = time.time()
                if self.ckpt is not None:
                    with HeartbeatTicker(self.env.rank, step, "saving", self._hb_tick):
                        self.ckpt.save(step, client_state={"step": step, "preempted": True,
                                                              "global_batch": self.global_batch}, blocking=True)
                self._say(f"preemption: emergency checkpoint at step {step} in {time.time() - t0:.2f}s; exiting")
                if self.ckpt is not None and self.ckpt.history:
                    self._say("emergency checkpoint record: " + json.dumps(json_safe(self.ckpt.history[-1])))
                rc = EXIT_PREEMPTED
                break
        if prev is not None and rc == 0:
            stop = self._decide(self._report(*prev), last)
            rc = stop or 0
        if rc == 0 and self.preempt and self.env.world == 1:
            # a notice that arrived after the last step was queued (one rank: no agreement needed)
            if self.ckpt is not None:
                with HeartbeatTicker(self.env.rank, last, "saving", self._hb_tick):
                    self.ckpt.save(last, client_state={"step": last, "preempted": True,
                                                          "global_batch": self.global_batch}, blocking=True)
            rc = EXIT_PREEMPTED
        if self.env.device.type == "cuda":
            dv = self.env.device
            self._say("memory: " + json.dumps({
                "peak_allocated_GiB": round(torch.cuda.max_memory_allocated(dv) / 2 ** 30, 1),
                "peak_reserved_GiB": round(torch.cuda.max_memory_reserved(dv) / 2 ** 30, 1),
                "alloc_retries": int(torch.cuda.memory_stats(dv).get("num_alloc_retries", 0)),
                "hbm_GiB": round(torch.cuda.get_device_properties(dv).total_memory / 2 ** 30, 1)}))
        if self.ckpt is not None:
            with HeartbeatTicker(self.env.rank, last, "finishing", self._hb_tick):
                self.ckpt.wait()
            if self.ckpt.prep_stats:
                ps = dict(self.ckpt.prep_stats)
                t0 = ps.pop("started_at", None)
                if t0 is not None and "done_at" in ps:
                    ps["done_after_start_s"] = round(ps.pop("done_at") - t0, 2)
                    ps["started_after_process_s"] = round(t0 - self.timeline["process_start"], 2)
                self._say("ckpt prepare: " + json.dumps(ps))
            if rc == 0 and a.export:
                with HeartbeatTicker(self.env.rank, last, "finishing", self._hb_tick):
                    export_consolidated(self.engine, a.export)
            # a finished job has nothing to resume: give the host RAM of the shm snapshot tier back
            self.ckpt.close(discard_shm=rc == 0)
        self.trap.close()
        self.pusher.close()
        telem = self.telemetry.stop() if self.telemetry is not None else None
        if telem is not None:
            self._say(f"telemetry: {json.dumps(telem)}")
        if a.log_json and self.env.rank == 0:
            with open(a.log_json, "w") as f:
                json.dump(json_safe({"log": self.log, "ckpt": self.ckpt.history if self.ckpt else [],
                                     "telemetry": telem,
                                     "trap": self.trap.records, "monitor": self.monitor.get_summary(),
                                     "engine": {"zero_stage": self.ecfg.zero_stage, "world": self.env.world,
                                                "backend": self.env.backend, "device": str(self.env.device),
                                                "notes": self.notes}}), f)
        if getattr(a, "dump_state", None):
            # per-rank outcome for multi-rank drills: exit code, last step read, this rank's fp32 partition
            os.makedirs(a.dump_state, exist_ok=True)
            self.engine.join_optimizer()
            torch.save({"rc": rc, "rank": self.env.rank, "last_step": self.log[-1]["step"] if self.log else start,
                        "step_count": self.engine.step_count, "master": self.engine.master.detach().cpu().clone()},
                       os.path.join(a.dump_state, f"rank{self.env.rank}.pt"))
        if torch.distributed.is_initialized():
            torch.distributed.destroy_process_group()
        return rc


def parse_args(argv=None) -> argparse.Namespace:
    ap = argparse.ArgumentParser(description="MI355X ZeRO training (DeepSpeed-config compatible)")
    ap.add_argument("--deepspeed_config", "--deepspeed-config", default=None)
    ap.add_argument("--model", default="llama-tiny")
    ap.add_argument("--seq-len", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--device", default="auto")
    ap.add_argument("--zero-stage", type=int, default=3)
    ap.add_argument("--fp16", action="store_true",
                    help="fp16 compute with the dynamic loss scaler (without a DeepSpeed config; else its fp16 block)")
    ap.add_argument("--micro-batch", type=int, default=1)
    ap.add_argument("--grad-accum", type=int, default=1)
    ap.add_argument("--auto-micro-batch", action="store_true",
                    help="size the micro-batch to the per-rank HBM plan (keeps micro-batch x grad-accum x world)")
    ap.add_argument("--lr", type=float, default=3e-4)
    ap.add_argument("--lr-scale", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--save-dir", default=None)
    ap.add_argument("--save-interval", type=int, default=0)
    ap.add_argument("--ckpt-mode", default="auto", choices=["auto", "device", "host", "shm"])
    ap.add_argument("--ckpt-shm", default="auto", choices=["auto", "on", "off"],
                    help="/dev/shm snapshot tier (outlives a SIGKILLed rank; restored first on auto-resume)")
    ap.add_argument("--ckpt-disk", type=int, default=1, help="0: snapshot tier only, no disk tags")
    ap.add_argument("--keep-last", type=int, default=3, help="complete disk tags kept")
    ap.add_argument("--elastic", action="store_true",
                    help="keep the first launch's global batch across restarts at other world sizes")
    ap.add_argument("--resume", default="none")
    ap.add_argument("--export", default=None, help="consolidated bf16 safetensors at the end (16-bit gather on save)")
    ap.add_argument("--inject-nan-step", type=int, default=-1)
    ap.add_argument("--kill-at-step", type=int, default=-1, help="fault drill: SIGKILL this rank after the step "
                    "(first attempt only)")
    ap.add_argument("--kill-rank", type=int, default=0, help="rank the SIGKILL drill kills")
    ap.add_argument("--stop-at-step", type=int, default=-1, help="hang drill: SIGSTOP this rank after the step "
                    "(first attempt only)")
    ap.add_argument("--stop-rank", type=int, default=0, help="rank the hang drill freezes")
    ap.add_argument("--preempt-at-step", type=int, default=-1, help="spot drill: deliver SIGUSR1 after the step")
    ap.add_argument("--preempt-when-ready", action="store_true",
                    help="spot drill: deliver the notice at the first step >= --preempt-at-step at which the "
                         "checkpoint snapshot buffer is prepared")
    ap.add_argument("--halt-on-nan", type=int, default=1)
    ap.add_argument("--metrics-url", default=os.environ.get("DLGM_METRICS_URL"))
    ap.add_argument("--job-id", default=os.environ.get("DLGM_JOB_ID", "local"))
    ap.add_argument("--log-interval", type=int, default=1)
    ap.add_argument("--telemetry-interval", type=float, default=5.0,
                    help="seconds between amdsmi samples of this rank's GPU (0: off)")
    ap.add_argument("--log-json", default=None)
    ap.add_argument("--n-layers", type=int, default=0, help="override the preset's depth (drills only)")
    ap.add_argument("--wall-clock-breakdown", action="store_true", help="per-phase HIP-event timers in the log")
    ap.add_argument("--expert-parallel", type=int, default=0, help="expert-parallel size (Mixtral)")
    ap.add_argument("--profile-steps", type=int, default=0, help="torch.profiler trace of N steps (from step 2)")
    ap.add_argument("--profile-dir", default="torch_trace")
    ap.add_argument("--sequence-parallel", type=int, default=0,
                    help="Ulysses sequence-parallel size: ranks of a group split each sequence")
    ap.add_argument("--hip-graphs", action="store_true",
                    help="replay each step's micro-batch loop as one captured HIP graph (single rank, dense)")
    ap.add_argument("--xgmi-mesh", default=None, choices=["on", "off"],
                    help="ZeRO gathers / reduce-scatters and the EP exchange over the device-driven xGMI mesh")
    ap.add_argument("--inject-nan-rank", type=int, default=-1,
                    help="with --inject-nan-step: poison the gradient on this rank only (-1: every rank)")
    ap.add_argument("--preempt-rank", type=int, default=-1,
                    help="with --preempt-at-step: deliver the preemption notice to this rank only (-1: every rank)")
    ap.add_argument("--shadow-world", type=int, default=0,
                    help="simulate rank --shadow-rank of a job of this many ranks alone on one GPU (true-size state)")
    ap.add_argument("--shadow-rank", type=int, default=0)
    ap.add_argument("--activation-checkpointing", action="store_true", help="block recompute in the backward")
    ap.add_argument("--dump-state", default=None, help="directory: each rank saves rc / last step / its partition")
    a, unknown = ap.parse_known_args(argv)
    return a


def main(argv=None) -> int:
    return Trainer(parse_args(argv)).run()
