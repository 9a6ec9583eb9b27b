"""Job registry + per-job supervisor: process ownership, log draining, heartbeat, auto-resume, MTTR.

The reference starts ``deepspeed`` with ``subprocess.Popen(stdout=PIPE, stderr=PIPE)``
and drops the handle (``ai_engine/deepspeed_launcher.py:354-362``): no registry, no
exit code, pipes never drained (the child blocks once ~64 KiB of output accumulate)
and the README's auto-resume claim (``README.md:14``) has no implementation. Here:

* every job runs in its own process group (``start_new_session``) so the whole rank
  tree can be signalled (spot notice -> SIGUSR1, cancel -> SIGTERM/SIGKILL);
* stdout/stderr go to ``<run_dir>/job.log`` (no pipes to fill up);
* the training ranks publish progress to ``<run_dir>/status.json`` (``DLGM_STATUS_FILE``, rank 0) and EVERY
  rank writes its own heartbeat to ``<run_dir>/heartbeat/rank{r}.json`` (``DLGM_HEARTBEAT_DIR``) after each
  completed step. Hang detection is on by default: a rank whose heartbeat is older than
  max(``heartbeat_min_s``, ``heartbeat_step_mult`` x the slowest rank's steady step time) -- or that never beat
  within ``startup_timeout_s`` of the attempt's start -- marks the attempt hung (a SIGSTOPped rank, a deadlocked
  collective: the others block in their next collective, so their beats go stale too; the stalest rank is named in
  the event). The whole rank tree is killed and the job resumes from the newest verified checkpoint. The ranks'
  process-group timeout (``DLGM_PG_TIMEOUT_S``) is set to the same bound, so a collective that can never complete
  also fails inside the rank;
* on a non-zero exit (SIGKILL'd rank, hang) the supervisor relaunches the job with
  ``--resume=auto`` (the engine rolls back to the newest checkpoint -- /dev/shm snapshot
  tier first -- that verifies on every rank) up to ``max_restarts`` times, and records
  MTTR = time of the first completed step after the restart - time the failure was
  detected;
* a NaN halt (exit code 3) is retried ``max_nan_restarts`` times with the learning rate
  scaled by ``nan_lr_backoff`` (the loss monitor's remediation, ``loss_monitor.py:135``:
  "Restore from last checkpoint and retry with lower LR"); the same data would otherwise
  hit the same NaN again, so a repeated halt ends the job as ``nan_halt``;
* elastic jobs (``elastic=True``; DeepSpeed ``elasticity`` block, reference
  ``deepspeed_launcher.py:78, 226-238``) relaunch at the largest world size that fits the
  healthy GPUs and divides the global batch; the trainer rescales gradient accumulation and
  the checkpoint reshards (``ckpt.checkpoint.ShardSource``).
"""
from __future__ import annotations

import json
import os
import signal
import subprocess
import tempfile
import threading
import time
from dataclasses import asdict, dataclass, field
from typing import Dict, List, Optional

EXIT_NAN_HALT = 3
EXIT_PREEMPTED = 4
EXIT_TRANSPORT = 5  # an xGMI mesh wait timed out (a peer died or stalled): resumed like a crash
# an EP routing overflowed an explicit ep_capacity_factor: a deterministic configuration error -- the resumed job would
# replay the same routing and overflow again, so it is not auto-resumed
EXIT_EP_OVERFLOW = 6


@dataclass
class JobSpec:
    job_id: str
    argv: List[str]
    env: Dict[str, str] = field(default_factory=dict)
    auto_resume: bool = True
    max_restarts: int = 3
    save_dir: Optional[str] = None
    run_dir: Optional[str] = None
    # hang detection: < 0 = auto (max(heartbeat_min_s, heartbeat_step_mult x steady step time)), 0 = off, > 0 fixed
    heartbeat_timeout_s: float = -1.0
    heartbeat_min_s: float = 120.0
    heartbeat_step_mult: float = 10.0
    startup_timeout_s: float = 900.0  # no heartbeat from some rank this long after an attempt started -> hung
    resume_arg: str = "--resume=auto"
    restart_on_preempt: bool = False
    max_nan_restarts: int = 1
    nan_lr_backoff: float = 0.5
    # elastic relaunch: world sizes in [min_world, max_world] with global_batch % (micro_batch * w) == 0
    elastic: bool = False
    min_world: int = 1
    max_world: int = 0
    global_batch: int = 0
    micro_batch: int = 1
    # /dev/shm snapshot tier owned by the supervisor: before the first launch, reserve this many
    # bytes of every local rank's snapshot file (ckpt/checkpoint.py reserve_snapshot_files), kept across restarts
    shm_reserve_bytes: int = 0
    shm_reserve_ranks: Optional[List[int]] = None


def _arg(argv: List[str], key: str) -> Optional[str]:
    for i, a in enumerate(argv):
        if a == key and i + 1 < len(argv):
            return argv[i + 1]
        if a.startswith(key + "="):
            return a.split("=", 1)[1]
    return None


def planned_snapshot_bytes(argv: List[str], nproc: Optional[int]) -> int:
    """Per-rank snapshot bytes of a training command (train.py options: --model, --zero-stage, --expert-parallel,
    --n-layers, --shadow-world), from the planner; 0 when the command does not say enough."""
    model = _arg(argv, "--model")
    if not model:
        return 0
    try:
        from ..models import get_config
        from ..parallel.planner import snapshot_bytes
        nl = int(_arg(argv, "--n-layers") or 0)
        m = get_config(model, **({"n_layers": nl} if nl else {}))
        world = int(_arg(argv, "--shadow-world") or 0) or (nproc or 1)
        return snapshot_bytes(m, world=world, zero_stage=int(_arg(argv, "--zero-stage") or 3),
                              ep_size=int(_arg(argv, "--expert-parallel") or 1))
    except (KeyError, ValueError):
        return 0


class Job:
    def __init__(self, spec: JobSpec):
        self.spec = spec
        self.run_dir = spec.run_dir or os.path.join(tempfile.gettempdir(), "dlgm_jobs", spec.job_id)
        os.makedirs(self.run_dir, exist_ok=True)
        self.log_path = os.path.join(self.run_dir, "job.log")
        self.status_path = os.path.join(self.run_dir, "status.json")
        self.heartbeat_dir = os.path.join(self.run_dir, "heartbeat")
        self.status = "pending"
        self.pid: Optional[int] = None
        self.restarts = 0
        self.exit_codes: List[int] = []
        self.events: List[Dict] = []
        self.mttr_s: List[float] = []
        self.world_history: List[int] = []
        self.nan_halts = 0
        self.lr_scale = 1.0
        self.created = time.time()
        self.ended: Optional[float] = None
        self._proc: Optional[subprocess.Popen] = None
        self._cancel = threading.Event()
        self._lock = threading.Lock()

    def event(self, kind: str, **kw) -> None:
        with self._lock:
            self.events.append({"t": time.time(), "event": kind, **kw})

    def progress(self) -> Optional[Dict]:
        try:
            with open(self.status_path) as f:
                return json.load(f)
        except (OSError, ValueError):
            return None

    def heartbeats(self) -> Dict[int, Dict]:
        """rank -> its last heartbeat record (every attempt's; callers filter on ``restart``)."""
        out: Dict[int, Dict] = {}
        try:
            names = os.listdir(self.heartbeat_dir)
        except OSError:
            return out
        for n in names:
            if n.startswith("rank") and n.endswith(".json"):
                try:
                    with open(os.path.join(self.heartbeat_dir, n)) as f:
                        rec = json.load(f)
                    out[int(n[4:-5])] = rec
                except (OSError, ValueError):
                    continue
        return out

    def to_dict(self) -> Dict:
        return {
            "job_id": self.spec.job_id, "status": self.status, "pid": self.pid, "restarts": self.restarts,
            "exit_codes": list(self.exit_codes), "log_path": self.log_path, "run_dir": self.run_dir,
            "mttr_s": list(self.mttr_s), "events": list(self.events[-50:]), "progress": self.progress(),
            "world_history": list(self.world_history), "nan_halts": self.nan_halts, "lr_scale": self.lr_scale,
            "command": self.spec.argv, "created": self.created, "ended": self.ended,
        }


class Supervisor(threading.Thread):
    def __init__(self, job: Job, poll_s: float = 0.2, first_proc: Optional[subprocess.Popen] = None):
        super().__init__(daemon=True, name=f"supervisor-{job.spec.job_id}")
        self.job = job
        self.poll_s = poll_s
        self._first = first_proc

    @staticmethod
    def nproc_of(argv: List[str]) -> Optional[int]:
        for i, a in enumerate(argv):
            for key in ("--nproc-per-node", "--nproc_per_node"):
                if a == key and i + 1 < len(argv):
                    return int(argv[i + 1])
                if a.startswith(key + "="):
                    return int(a.split("=", 1)[1])
        return None

    @staticmethod
    def with_nproc(argv: List[str], n: int) -> List[str]:
        out = list(argv)
        for i, a in enumerate(out):
            for key in ("--nproc-per-node", "--nproc_per_node"):
                if a == key and i + 1 < len(out):
                    out[i + 1] = str(n)
                    return out
                if a.startswith(key + "="):
                    out[i] = f"{key}={n}"
                    return out
        raise ValueError("elastic job argv has no --nproc-per-node")

    def available_world(self, current: int) -> int:
        """Ranks the next attempt can use: an operator / health monitor may write the count to
        <run_dir>/available_world; otherwise one GPU is assumed lost with the failed rank."""
        p = os.path.join(self.job.run_dir, "available_world")
        try:
            with open(p) as f:
                return int(f.read().strip())
        except (OSError, ValueError):
            return max(1, current - 1)

    def elastic_world(self, current: int) -> int:
        spec = self.job.spec
        avail = min(self.available_world(current), spec.max_world or current)
        gb = spec.global_batch or 0
        for w in range(avail, spec.min_world - 1, -1):
            if not gb or gb % (spec.micro_batch * w) == 0:
                return w
        return 0

    def heartbeat_timeout(self, beats: Dict[int, Dict]) -> float:
        """Seconds without a heartbeat after which a rank is hung (0: detection off)."""
        spec = self.job.spec
        if spec.heartbeat_timeout_s >= 0:
            return spec.heartbeat_timeout_s
        step_s = max([float(b.get("step_s") or 0.0) for b in beats.values()] or [0.0])
        return max(spec.heartbeat_min_s, spec.heartbeat_step_mult * step_s)

    def hung_rank(self, attempt_t0: float, expected: Optional[int], now: Optional[float] = None) -> Optional[Dict]:
        """The stalest rank of the current attempt if it is past its bound, else None."""
        job, spec = self.job, self.job.spec
        now = time.time() if now is None else now
        beats = {r: b for r, b in job.heartbeats().items() if b.get("restart", 0) == job.restarts
                 and b.get("time", 0) >= attempt_t0}
        prog = job.progress()
        if not beats and prog is not None and prog.get("restart", 0) == job.restarts and \
                prog.get("time", 0) >= attempt_t0:
            beats = {0: prog}  # a rank-0-only status writer (older training scripts)
        timeout = self.heartbeat_timeout(beats)
        if timeout <= 0:
            return None
        ranks = range(expected) if expected else sorted(beats)
        worst = None
        for r in ranks:
            b = beats.get(r)
            if b is None:  # never beat in this attempt: the startup bound (at least the steady-state one)
                age, bound = now - attempt_t0, max(spec.startup_timeout_s, timeout)
            elif b.get("phase") in BLOCKING_PHASES:
                # a blocking checkpoint write-out / export (engine/trainer.py HeartbeatTicker): the rank beats from a
                # ticker thread meanwhile, under the start-up bound; a block that outlasts BLOCK_LIMIT_MULT start-up
                # bounds is a hang even while the ticker runs (a deadlocked writer, a collective that never returns)
                bound = max(spec.startup_timeout_s, timeout)
                age = now - float(b.get("time", attempt_t0))
                since = float(b.get("blocked_since") or b.get("time", attempt_t0))
                if now - since > BLOCK_LIMIT_MULT * bound:
                    age, bound = now - since, BLOCK_LIMIT_MULT * bound
            elif not b.get("step_s") and spec.heartbeat_timeout_s < 0:
                # ready, no step finished yet (restore, warm-up, the first step): no step time to scale by
                age, bound = now - float(b.get("time", attempt_t0)), max(spec.startup_timeout_s, timeout)
            else:
                age, bound = now - float(b.get("time", attempt_t0)), timeout
            if age > bound and (worst is None or age > worst["age_s"]):
                worst = {"rank": r, "age_s": round(age, 2), "bound_s": round(bound, 2),
                         "last_step": None if b is None else b.get("step")}
        if worst is None and not expected and not beats and spec.heartbeat_timeout_s > 0 \
                and now - attempt_t0 > max(spec.startup_timeout_s, timeout):
            worst = {"rank": None, "age_s": round(now - attempt_t0, 2), "bound_s": spec.startup_timeout_s,
                     "last_step": None}
        return worst

    def expected_ranks(self) -> Optional[int]:
        argv = self.job.spec.argv
        n = self.nproc_of(argv)
        if self.job.world_history:
            n = self.job.world_history[-1]
        return n

    def _start(self, resume: bool) -> subprocess.Popen:
        spec = self.job.spec
        argv = list(spec.argv)
        if self.job.world_history and self.nproc_of(argv) is not None:
            argv = self.with_nproc(argv, self.job.world_history[-1])
        if resume and spec.resume_arg not in argv:
            argv.append(spec.resume_arg)
        if self.job.lr_scale != 1.0:
            argv += ["--lr-scale", str(self.job.lr_scale)]
        env = {**os.environ, **spec.env, "DLGM_STATUS_FILE": self.job.status_path, "DLGM_JOB_ID": spec.job_id,
               "DLGM_RESTART": str(self.job.restarts), "DLGM_HEARTBEAT_DIR": self.job.heartbeat_dir}
        if spec.heartbeat_timeout_s != 0:
            # a collective that can never complete fails inside the ranks on the same bound (the auto bound before
            # any step time is known: the startup one)
            pg = spec.heartbeat_timeout_s if spec.heartbeat_timeout_s > 0 else max(spec.heartbeat_min_s,
                                                                                  spec.startup_timeout_s)
            env.setdefault("DLGM_PG_TIMEOUT_S", str(int(max(30.0, pg))))
        os.makedirs(self.job.heartbeat_dir, exist_ok=True)
        if spec.save_dir:
            env["DLGM_SAVE_DIR"] = spec.save_dir
        log = open(self.job.log_path, "ab", buffering=0)
        try:
            proc = subprocess.Popen(argv, stdout=log, stderr=subprocess.STDOUT, env=env, start_new_session=True)
        finally:
            log.close()
        self.job.pid = proc.pid
        self.job._proc = proc
        self.job.status = "running"
        self.job.event("started", pid=proc.pid, resume=resume)
        return proc

    def _kill_group(self, proc: subprocess.Popen, grace_s: float = 10.0) -> None:
        try:
            os.killpg(proc.pid, signal.SIGTERM)
        except ProcessLookupError:
            return
        t0 = time.time()
        while proc.poll() is None and time.time() - t0 < grace_s:
            time.sleep(0.05)
        if proc.poll() is None:
            try:
                os.killpg(proc.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            proc.wait()

    def reserve_shm(self) -> None:
        """The snapshot files of this node's ranks, reserved before the first launch and kept across restarts."""
        job, spec = self.job, self.job.spec
        if spec.shm_reserve_bytes <= 0 or not spec.save_dir:
            return
        from ..ckpt.checkpoint import reserve_snapshot_files
        ranks = spec.shm_reserve_ranks if spec.shm_reserve_ranks is not None else \
            list(range(self.nproc_of(spec.argv) or 1))
        try:
            rec = reserve_snapshot_files(spec.save_dir, ranks, spec.shm_reserve_bytes)
        except OSError as e:
            rec = {"error": str(e)}
        job.event("shm_reserved", bytes_per_rank=spec.shm_reserve_bytes, ranks=len(ranks), **rec)

    def run(self) -> None:
        job, spec = self.job, self.job.spec
        w0 = self.nproc_of(spec.argv)
        if w0 is not None:
            job.world_history.append(w0)
        if self._first is None:
            self.reserve_shm()
        proc = self._first if self._first is not None else self._start(resume=False)
        failure_t: Optional[float] = None
        step_at_failure = -1
        attempt_t0 = time.time()
        while True:
            rc = proc.poll()
            prog = job.progress()
            if failure_t is not None and prog and prog.get("step", -1) > step_at_failure and \
                    prog.get("restart", 0) == job.restarts and prog.get("time", 0) >= failure_t:
                job.mttr_s.append(prog["time"] - failure_t)
                job.event("recovered", mttr_s=job.mttr_s[-1], step=prog.get("step"))
                failure_t = None
            # heartbeat: only records of the current attempt count, measured from the attempt start
            hung = self.hung_rank(attempt_t0, self.expected_ranks()) if rc is None else None
            if hung is not None:
                job.event("heartbeat_lost", **hung)
                self._kill_group(proc, grace_s=2.0)
                rc = proc.poll() if proc.poll() is not None else -9
            if job._cancel.is_set():
                self._kill_group(proc)
                job.status = "cancelled"
                break
            if rc is None:
                time.sleep(self.poll_s)
                continue
            job.exit_codes.append(rc)
            job.event("exited", rc=rc)
            if rc == 0:
                job.status = "succeeded"
                break
            preempted = rc == EXIT_PREEMPTED
            if preempted and not spec.restart_on_preempt:
                job.status = "preempted"
                break
            if rc == EXIT_EP_OVERFLOW:
                job.status = "failed"
                job.event("ep_capacity_overflow", hint="raise mi355x.ep_capacity_factor or use the dropless default")
                break
            nan = rc == EXIT_NAN_HALT
            if nan:
                job.nan_halts += 1
                if job.nan_halts > spec.max_nan_restarts:
                    job.status = "nan_halt"
                    job.event("nan_halt", halts=job.nan_halts)
                    break
                job.lr_scale *= spec.nan_lr_backoff
            if spec.auto_resume and job.restarts < spec.max_restarts:
                # make sure no straggler rank of the failed attempt survives
                try:
                    os.killpg(proc.pid, signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass
                failure_t = time.time()
                step_at_failure = (prog or {}).get("step", -1)
                if spec.elastic and not nan and job.world_history:
                    w = self.elastic_world(job.world_history[-1])
                    if w < 1:
                        job.status = "failed"
                        job.event("elastic_no_valid_world", last=job.world_history[-1])
                        break
                    job.world_history.append(w)
                job.restarts += 1
                job.status = "restarting"
                job.event("restarting", attempt=job.restarts, reason="nan_halt" if nan else "crash",
                          world=job.world_history[-1] if job.world_history else None, lr_scale=job.lr_scale)
                proc = self._start(resume=True)
                attempt_t0 = time.time()
                continue
            job.status = "failed"
            break
        job.ended = time.time()


class JobRegistry:
    """Thread-safe registry of supervised jobs (process-global via :func:`default_registry`)."""

    def __init__(self):
        self._jobs: Dict[str, Job] = {}
        self._lock = threading.Lock()

    def submit(self, spec: JobSpec) -> Job:
        job = Job(spec)
        # start the first attempt synchronously so launch errors (missing binary) surface to the caller -- after the
        # shm snapshot files are reserved (Supervisor.run skips that for a job whose first attempt is already running)
        first = Supervisor(job)
        first.reserve_shm()
        proc = first._start(resume=False)
        sup = Supervisor(job, first_proc=proc)
        with self._lock:
            self._jobs[spec.job_id] = job
        sup.start()
        return job

    def get(self, job_id: str) -> Optional[Job]:
        with self._lock:
            return self._jobs.get(job_id)

    def list(self) -> List[Job]:
        with self._lock:
            return list(self._jobs.values())

    def cancel(self, job_id: str) -> bool:
        job = self.get(job_id)
        if job is None:
            return False
        job._cancel.set()
        return True

    def signal(self, job_id: str, sig: int) -> bool:
        job = self.get(job_id)
        if job is None or job.pid is None:
            return False
        try:
            os.killpg(job.pid, sig)
            return True
        except ProcessLookupError:
            return False


_DEFAULT: Optional[JobRegistry] = None


def default_registry() -> JobRegistry:
    global _DEFAULT
    if _DEFAULT is None:
        _DEFAULT = JobRegistry()
    return _DEFAULT


def _write_json(path: str, rec: Dict) -> None:
    tmp = f"{path}.{os.getpid()}.tmp"
    with open(tmp, "w") as f:
        json.dump(rec, f)
    os.replace(tmp, path)


def write_status(step: int, **kw) -> None:
    """Called by training rank 0 after each completed step (atomic replace)."""
    path = os.environ.get("DLGM_STATUS_FILE")
    if not path:
        return
    _write_json(path, {"step": step, "time": time.time(), "restart": int(os.environ.get("DLGM_RESTART", "0")), **kw})


# heartbeat phases written while a rank blocks outside the step loop (final checkpoint flush, export, emergency save)
BLOCKING_PHASES = ("saving", "finishing")
BLOCK_LIMIT_MULT = 4.0


def write_heartbeat(rank: int, step: int, **kw) -> None:
    """Called by EVERY training rank after each completed step (and once when it is ready to train): the
    supervisor's hang detection reads one file per rank (``DLGM_HEARTBEAT_DIR``)."""
    d = os.environ.get("DLGM_HEARTBEAT_DIR")
    if not d:
        return
    os.makedirs(d, exist_ok=True)
    _write_json(os.path.join(d, f"rank{int(rank)}.json"),
                {"rank": int(rank), "step": step, "time": time.time(), "pid": os.getpid(),
                 "restart": int(os.environ.get("DLGM_RESTART", "0")), **kw})


def main(argv: Optional[List[str]] = None) -> int:
    """``python -m ...launcher.supervisor [opts] -- <training command ...>``

    Runs the command under a :class:`Supervisor` in the foreground (container entry point / CLI);
    exits with the job's final code. SIGTERM/SIGINT cancel the job (the rank tree gets SIGTERM).
    """
    import argparse
    import sys

    argv = list(sys.argv[1:] if argv is None else argv)
    if "--" not in argv:
        print("usage: supervisor [--max-restarts N] [--job-id ID] [--run-dir D] [--save-dir D] "
              "[--heartbeat-timeout S] [--restart-on-preempt] -- <command ...>", file=sys.stderr)
        return 2
    cut = argv.index("--")
    ap = argparse.ArgumentParser(prog="supervisor")
    ap.add_argument("--max-restarts", type=int, default=3)
    ap.add_argument("--job-id", default=f"job_{int(time.time())}")
    ap.add_argument("--run-dir", default=None)
    ap.add_argument("--save-dir", default=None)
    ap.add_argument("--heartbeat-timeout", type=float, default=-1.0,
                    help="seconds without a rank heartbeat before the job is killed and resumed (-1: auto, 0: off)")
    ap.add_argument("--heartbeat-min", type=float, default=120.0)
    ap.add_argument("--startup-timeout", type=float, default=900.0)
    ap.add_argument("--restart-on-preempt", action="store_true")
    ap.add_argument("--no-auto-resume", action="store_true")
    ap.add_argument("--max-nan-restarts", type=int, default=1)
    ap.add_argument("--elastic", action="store_true", help="relaunch at a smaller world size after a rank failure")
    ap.add_argument("--min-world", type=int, default=1)
    ap.add_argument("--max-world", type=int, default=0)
    ap.add_argument("--global-batch", type=int, default=0)
    ap.add_argument("--micro-batch", type=int, default=1)
    ap.add_argument("--shm-reserve", default="off",
                    help="reserve the ranks' /dev/shm snapshot files before the first launch: 'auto' (planner size "
                         "from the training command), 'off', or GiB per rank")
    a = ap.parse_args(argv[:cut])
    cmd = argv[cut + 1:]
    shm_bytes = 0
    if a.shm_reserve == "auto":
        shm_bytes = planned_snapshot_bytes(cmd, Supervisor.nproc_of(cmd))
    elif a.shm_reserve != "off":
        shm_bytes = int(float(a.shm_reserve) * (1 << 30))
    spec = JobSpec(job_id=a.job_id, argv=cmd, auto_resume=not a.no_auto_resume, max_restarts=a.max_restarts,
                   save_dir=a.save_dir, run_dir=a.run_dir, heartbeat_timeout_s=a.heartbeat_timeout,
                   heartbeat_min_s=a.heartbeat_min, startup_timeout_s=a.startup_timeout,
                   restart_on_preempt=a.restart_on_preempt, max_nan_restarts=a.max_nan_restarts,
                   elastic=a.elastic, min_world=a.min_world, max_world=a.max_world, global_batch=a.global_batch,
                   micro_batch=a.micro_batch, shm_reserve_bytes=shm_bytes)
    job = Job(spec)
    sup = Supervisor(job)
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, lambda *_: job._cancel.set())
    sup.start()
    while sup.is_alive():
        sup.join(0.5)
    print(json.dumps(job.to_dict(), default=str), flush=True)
    if job.status == "succeeded":
        return 0
    return job.exit_codes[-1] if job.exit_codes and job.exit_codes[-1] > 0 else 1


if __name__ == "__main__":
    raise SystemExit(main())
