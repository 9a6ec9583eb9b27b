"""Hung-rank detection on the default launch path (reference watcher loop
``/root/reference/ai_engine/spot_resiliency.py:17-37``, auto-resume claim ``/root/reference/README.md:14``).

Every training rank writes its own heartbeat before it issues a step; the supervisor's bound is
max(heartbeat_min_s, 10 x the steady step time) once a step time is known, the start-up bound before. The drill
SIGSTOPs rank 2 of a 4-rank gloo job after step 3: the other ranks block in their next collective, the supervisor
names rank 2 as the stalest, kills the rank tree and relaunches at W = 4 from the newest verified tag."""
import json
import os
import socket
import sys
import time

import torch

from distributed_llm_training_gpu_manager_amd.launcher.config import DeepSpeedConfig, MI355XOptions
from distributed_llm_training_gpu_manager_amd.launcher.supervisor import Job, JobRegistry, JobSpec, Supervisor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _beat(d, rank, step, t, step_s=None, restart=0):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, f"rank{rank}.json"), "w") as f:
        json.dump({"rank": rank, "step": step, "time": t, "restart": restart, "step_s": step_s}, f)


def test_hung_rank_bounds(tmp_path):
    job = Job(JobSpec(job_id="hb", argv=["x", "--nproc-per-node", "4"], run_dir=str(tmp_path / "run"),
                      heartbeat_min_s=10.0, startup_timeout_s=100.0))
    sup = Supervisor(job)
    t0 = 1000.0
    # nobody beat yet: only the start-up bound applies
    assert sup.hung_rank(t0, 4, now=t0 + 50) is None
    assert sup.hung_rank(t0, 4, now=t0 + 101)["rank"] == 0
    # ranks 0, 1, 3 beat recently with a 2 s step time (bound = max(10, 10 x 2) = 20 s), rank 2 is 25 s old
    for r in (0, 1, 3):
        _beat(job.heartbeat_dir, r, 7, t0 + 60, step_s=2.0)
    _beat(job.heartbeat_dir, 2, 6, t0 + 50, step_s=2.0)
    assert sup.hung_rank(t0, 4, now=t0 + 65) is None
    h = sup.hung_rank(t0, 4, now=t0 + 75)
    assert h["rank"] == 2 and h["last_step"] == 6 and h["bound_s"] == 20.0
    # a beat without a step time (ready / first step): the start-up bound
    _beat(job.heartbeat_dir, 2, 6, t0 + 50, step_s=None)
    assert sup.hung_rank(t0, 4, now=t0 + 75) is None
    # records of an earlier attempt do not count; explicit 0 turns detection off
    job.restarts = 1
    assert sup.hung_rank(t0, 4, now=t0 + 99) is None  # the old beats are ignored: start-up bound again
    assert sup.hung_rank(t0, 4, now=t0 + 101)["rank"] == 0
    job.spec.heartbeat_timeout_s = 0.0
    assert sup.hung_rank(t0, 4, now=t0 + 10_000) is None


def test_launcher_enables_hang_detection_by_default():
    opts = MI355XOptions()
    assert opts.heartbeat_timeout_s < 0 and opts.heartbeat_min_s == 120.0  # auto bound, on
    cfg = DeepSpeedConfig(model_name="m", mi355x=opts)
    from distributed_llm_training_gpu_manager_amd.launcher.launcher import ZeroLauncher
    seen = {}

    class _Reg:
        def submit(self, spec):
            seen["spec"] = spec
            raise RuntimeError("not launching in this test")
    ZeroLauncher(registry=_Reg()).launch(cfg, "train.py")
    assert seen["spec"].heartbeat_timeout_s < 0 and seen["spec"].startup_timeout_s == 900.0


def test_sigstopped_rank_is_detected_and_job_resumes_at_full_world(tmp_path):
    argv = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "4", "--master-addr", "127.0.0.1",
            "--master-port", str(_port()), "-m", "distributed_llm_training_gpu_manager_amd.train", "--device", "cpu",
            "--zero-stage", "3", "--steps", "6", "--seq-len", "32", "--save-interval", "2", "--stop-at-step", "3",
            "--stop-rank", "2", "--ckpt-shm", "off", "--dump-state", str(tmp_path / "dump")]
    reg = JobRegistry()
    job = reg.submit(JobSpec(job_id="stop2", argv=argv, env={"PYTHONPATH": ROOT, "OMP_NUM_THREADS": "1"},
                             save_dir=str(tmp_path / "ck"), run_dir=str(tmp_path / "run"), max_restarts=2,
                             heartbeat_min_s=6.0, startup_timeout_s=90.0))
    t0 = time.time()
    while job.status not in ("succeeded", "failed", "nan_halt") and time.time() - t0 < 400:
        time.sleep(0.2)
    log = open(job.log_path).read()
    assert job.status == "succeeded", log[-4000:]
    lost = [e for e in job.events if e["event"] == "heartbeat_lost"]
    assert len(lost) == 1 and lost[0]["rank"] == 2, job.events
    # detected within the bound (6 s; steps on CPU take far less than 0.6 s) plus the supervisor's polling
    assert lost[0]["age_s"] < lost[0]["bound_s"] + 3.0, lost
    assert job.restarts == 1 and job.world_history[-1] == 4
    assert "resumed from step 2" in log
    d = [torch.load(os.path.join(tmp_path / "dump", f"rank{r}.pt"), weights_only=True) for r in range(4)]
    assert [x["rc"] for x in d] == [0] * 4 and all(x["step_count"] == 6 for x in d)


def test_blocking_phases_get_the_startup_bound_and_a_ticker(tmp_path, monkeypatch):
    """a rank blocked in the final checkpoint write-out / export beats from a ticker thread with
    phase 'saving' / 'finishing'; the supervisor gives those beats the start-up bound, and a block that outlasts
    BLOCK_LIMIT_MULT such bounds is still named hung (a deadlocked writer keeps ticking)."""
    from distributed_llm_training_gpu_manager_amd.engine.trainer import HeartbeatTicker
    from distributed_llm_training_gpu_manager_amd.launcher.supervisor import BLOCK_LIMIT_MULT

    job = Job(JobSpec(job_id="hb2", argv=["x", "--nproc-per-node", "1"], run_dir=str(tmp_path / "run"),
                      heartbeat_min_s=10.0, startup_timeout_s=100.0))
    sup = Supervisor(job)
    t0 = 1000.0
    d = job.heartbeat_dir
    os.makedirs(d, exist_ok=True)

    def beat(**kw):
        with open(os.path.join(d, "rank0.json"), "w") as f:
            json.dump({"rank": 0, "step": 9, "restart": 0, **kw}, f)
    # steady 2 s steps: the bound is 20 s; a 'finishing' beat 60 s old is within the 100 s start-up bound
    beat(time=t0 + 10, phase="finishing", blocked_since=t0 + 10)
    assert sup.hung_rank(t0, 1, now=t0 + 70) is None
    assert sup.hung_rank(t0, 1, now=t0 + 120)["rank"] == 0  # the ticker died: past the start-up bound
    # a ticker still beating, but blocked for longer than BLOCK_LIMIT_MULT start-up bounds
    beat(time=t0 + 500, phase="saving", blocked_since=t0 + 200)
    assert sup.hung_rank(t0, 1, now=t0 + 501) is None
    beat(time=t0 + 600, phase="saving", blocked_since=t0 + 200)
    h = sup.hung_rank(t0, 1, now=t0 + 200 + BLOCK_LIMIT_MULT * 100 + 1)
    assert h is not None and h["bound_s"] == BLOCK_LIMIT_MULT * 100

    # the ticker itself: fresh beats while the body blocks, phase and blocked_since recorded
    monkeypatch.setenv("DLGM_HEARTBEAT_DIR", str(tmp_path / "hb"))
    path = tmp_path / "hb" / "rank3.json"
    with HeartbeatTicker(3, 41, "finishing", interval_s=0.1):
        first = json.loads(path.read_text())
        time.sleep(0.35)
        later = json.loads(path.read_text())
    assert first["phase"] == later["phase"] == "finishing" and first["step"] == 41
    assert later["time"] > first["time"] and later["blocked_since"] == first["blocked_since"]
