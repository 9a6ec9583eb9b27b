"""Job supervisor: log draining, exit codes, auto-resume with MTTR, cancel, heartbeat loss."""
import json
import os
import sys
import textwrap
import time

from distributed_llm_training_gpu_manager_amd.launcher.supervisor import JobRegistry, JobSpec


def _script(tmp_path, body: str) -> str:
    p = tmp_path / "job.py"
    p.write_text(textwrap.dedent(body))
    return str(p)


FAKE_TRAIN = """
import json, os, sys, time
resume = "--resume=auto" in sys.argv
state = os.path.join(os.path.dirname(os.environ["DLGM_STATUS_FILE"]), "ckpt_step")
start = int(open(state).read()) if resume and os.path.exists(state) else 0
for step in range(start + 1, 7):
    time.sleep(0.05)
    open(state, "w").write(str(step))
    from distributed_llm_training_gpu_manager_amd.launcher.supervisor import write_status
    write_status(step, loss=1.0 / step)
    print("step", step, flush=True)
    if step == 3 and not resume:
        os.kill(os.getpid(), 9)   # mid-run SIGKILL
sys.exit(0)
"""


def _wait(job, states, timeout=30):
    t0 = time.time()
    while job.status not in states and time.time() - t0 < timeout:
        time.sleep(0.05)
    return job.status


def test_sigkill_auto_resume_measures_mttr(tmp_path):
    reg = JobRegistry()
    env = {"PYTHONPATH": os.path.dirname(os.path.dirname(os.path.abspath(__file__)))}
    job = reg.submit(JobSpec(job_id="j1", argv=[sys.executable, _script(tmp_path, FAKE_TRAIN)], env=env,
                             run_dir=str(tmp_path / "run")))
    assert _wait(job, ("succeeded", "failed")) == "succeeded", open(job.log_path).read()
    assert job.restarts == 1 and job.exit_codes[0] == -9 and job.exit_codes[-1] == 0
    assert len(job.mttr_s) == 1 and 0 < job.mttr_s[0] < 20
    log = open(job.log_path).read()
    assert "step 3" in log and "step 6" in log  # drained to file, resumed after step 3
    assert any(e["event"] == "recovered" for e in job.to_dict()["events"])


def test_failure_without_resume_and_cancel(tmp_path):
    reg = JobRegistry()
    job = reg.submit(JobSpec(job_id="j2", argv=[sys.executable, "-c", "import sys; sys.exit(5)"], auto_resume=False,
                             run_dir=str(tmp_path / "r2")))
    assert _wait(job, ("failed",)) == "failed" and job.exit_codes == [5]
    job3 = reg.submit(JobSpec(job_id="j3", argv=[sys.executable, "-c", "import time; time.sleep(60)"],
                              run_dir=str(tmp_path / "r3")))
    time.sleep(0.3)
    assert reg.cancel("j3")
    assert _wait(job3, ("cancelled",)) == "cancelled"


def test_heartbeat_loss_triggers_restart(tmp_path):
    reg = JobRegistry()
    body = """
    import os, sys, time
    from distributed_llm_training_gpu_manager_amd.launcher.supervisor import write_status
    write_status(1)
    if "--resume=auto" not in sys.argv:
        time.sleep(60)   # hang
    write_status(2)
    """
    env = {"PYTHONPATH": os.path.dirname(os.path.dirname(os.path.abspath(__file__)))}
    job = reg.submit(JobSpec(job_id="j4", argv=[sys.executable, _script(tmp_path, body)], env=env,
                             heartbeat_timeout_s=1.0, run_dir=str(tmp_path / "r4")))
    assert _wait(job, ("succeeded", "failed")) == "succeeded"
    assert job.restarts == 1 and any(e["event"] == "heartbeat_lost" for e in job.events)


def test_supervisor_cli_restarts_then_succeeds(tmp_path):
    """CLI entry point (infra/train-job.yaml): a command failing once is resumed and succeeds."""
    import subprocess
    import sys

    marker = tmp_path / "failed_once"
    script = tmp_path / "flaky.py"
    script.write_text(
        "import os, sys\n"
        f"m = {str(marker)!r}\n"
        "if not os.path.exists(m):\n"
        "    open(m, 'w').close(); sys.exit(7)\n"
        "assert '--resume=auto' in sys.argv\n")
    r = subprocess.run([sys.executable, "-m", "distributed_llm_training_gpu_manager_amd.launcher.supervisor",
                        "--max-restarts", "2", "--run-dir", str(tmp_path / "run"), "--",
                        sys.executable, str(script)], capture_output=True, text=True, timeout=120,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stderr
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["status"] == "succeeded" and rec["restarts"] == 1 and rec["exit_codes"] == [7, 0]


def test_ep_capacity_overflow_is_not_resumed(tmp_path):
    """an EP overflow of an explicit capacity (exit 6) replays identically on resume: it fails the job at
    once, while a mesh timeout (exit 5) is resumed like a crash."""
    from distributed_llm_training_gpu_manager_amd.launcher.supervisor import EXIT_EP_OVERFLOW, EXIT_TRANSPORT
    reg = JobRegistry()
    job = reg.submit(JobSpec(job_id="ovf", argv=[sys.executable, "-c", f"import sys; sys.exit({EXIT_EP_OVERFLOW})"],
                             run_dir=str(tmp_path / "r1"), max_restarts=3))
    assert _wait(job, ("failed", "succeeded")) == "failed" and job.exit_codes == [EXIT_EP_OVERFLOW]
    assert job.restarts == 0 and any(e["event"] == "ep_capacity_overflow" for e in job.to_dict()["events"])
    job2 = reg.submit(JobSpec(job_id="tmo", argv=[sys.executable, "-c", f"import sys; sys.exit({EXIT_TRANSPORT})"],
                              run_dir=str(tmp_path / "r2"), max_restarts=1))
    assert _wait(job2, ("failed", "succeeded")) == "failed"
    assert job2.restarts == 1 and job2.exit_codes == [EXIT_TRANSPORT, EXIT_TRANSPORT]
