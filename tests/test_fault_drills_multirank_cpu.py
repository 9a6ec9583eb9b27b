"""Multi-rank fault drills (BASELINE configs 3-5 at W = 4, gloo on CPU): ONE faulty rank among healthy ones.

The reference's spot manager is meant to save "a distributed checkpoint" on a notice
(``/root/reference/ai_engine/spot_resiliency.py:8-10, 43-49``) and its README promises auto-resume
(``/root/reference/README.md:14``); config 3 halts an 8-GPU job on NaN. Each drill launches the real trainer under
``torch.distributed.run`` with 4 ranks and injects the fault on one rank only:

* NaN in rank 2's gradient at step 3 -> the non-finite count rides the all-reduced gradient statistics, every rank
  skips the update on the device (NaN latch) and exits 3 at the same step, each holding its pre-NaN partition;
* preemption notice on rank 1 only (Mixtral-tiny, EP = 4) -> the flag rides the next step's statistics, every rank
  writes the same emergency tag and exits 4; a relaunch at W = 4 resumes at the next step;
* SIGKILL of rank 3 -> the supervisor tears the job down and relaunches at W = 4 from the newest verified tag.
"""
import os
import socket
import subprocess
import sys
import time

import torch

from distributed_llm_training_gpu_manager_amd.ckpt.checkpoint import complete_tags
from distributed_llm_training_gpu_manager_amd.launcher.supervisor import (EXIT_NAN_HALT, EXIT_PREEMPTED,
                                                                         JobRegistry, JobSpec)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = {**os.environ, "PYTHONPATH": ROOT, "OMP_NUM_THREADS": "1"}


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(n, *args, timeout=420):
    argv = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
            "--master-port", str(_port()), "-m", "distributed_llm_training_gpu_manager_amd.train", "--device", "cpu",
            "--seq-len", "32", "--log-interval", "100", *args]
    return subprocess.run(argv, env=ENV, capture_output=True, text=True, timeout=timeout)


def _dumps(d, n):
    return [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(n)]


def test_nan_on_one_rank_halts_every_rank_at_the_same_step(tmp_path):
    ref = tmp_path / "ref"
    r = _torchrun(4, "--zero-stage", "3", "--steps", "2", "--dump-state", str(ref))
    assert r.returncode == 0, r.stderr[-3000:]
    got = tmp_path / "nan"
    r = _torchrun(4, "--zero-stage", "3", "--steps", "6", "--inject-nan-step", "3", "--inject-nan-rank", "2",
                  "--dump-state", str(got))
    d, want = _dumps(got, 4), _dumps(ref, 4)
    assert [x["rc"] for x in d] == [EXIT_NAN_HALT] * 4, (r.stdout[-2000:], r.stderr[-3000:])
    assert [x["last_step"] for x in d] == [3] * 4
    for x, w in zip(d, want):  # every rank kept the state before the poisoned step (and the step queued after it)
        assert torch.equal(x["master"], w["master"]), x["rank"]


def test_preemption_notice_on_one_rank_saves_one_tag_everywhere(tmp_path):
    save = tmp_path / "ck"
    common = ["--model", "mixtral-tiny", "--expert-parallel", "4", "--zero-stage", "3", "--save-dir", str(save),
              "--ckpt-shm", "off"]
    r = _torchrun(4, *common, "--steps", "10", "--preempt-at-step", "4", "--preempt-rank", "1",
                  "--dump-state", str(tmp_path / "pre"))
    d = _dumps(tmp_path / "pre", 4)
    assert [x["rc"] for x in d] == [EXIT_PREEMPTED] * 4, (r.stdout[-2000:], r.stderr[-3000:])
    tags = complete_tags(str(save))
    assert len(tags) == 1, tags
    k = int(tags[0].replace("global_step", ""))
    # the notice arrives after step 4 on rank 1; its flag rides step 5's all-reduced statistics, which every rank reads
    # while step 6 is already queued (one-step-behind host reads): all ranks checkpoint step 6 and stop
    assert k == 6, k
    assert all(x["step_count"] == d[0]["step_count"] for x in d)
    r = _torchrun(4, *common, "--steps", str(k + 2), "--resume", "auto", "--dump-state", str(tmp_path / "post"))
    post = _dumps(tmp_path / "post", 4)
    assert [x["rc"] for x in post] == [0] * 4, r.stderr[-3000:]
    assert f"resumed from step {k}" in r.stdout, r.stdout[-2000:]
    assert all(x["step_count"] == k + 2 for x in post)


def test_sigkill_of_one_rank_resumes_at_full_world(tmp_path):
    port = _port()
    argv = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "4", "--master-addr", "127.0.0.1",
            "--master-port", str(port), "-m", "distributed_llm_training_gpu_manager_amd.train", "--device", "cpu",
            "--zero-stage", "3", "--steps", "6", "--seq-len", "32", "--save-interval", "2", "--kill-at-step", "3",
            "--kill-rank", "3", "--ckpt-shm", "off", "--dump-state", str(tmp_path / "dump")]
    reg = JobRegistry()
    job = reg.submit(JobSpec(job_id="kill3", argv=argv, env={"PYTHONPATH": ROOT, "OMP_NUM_THREADS": "1"},
                             save_dir=str(tmp_path / "ck"), run_dir=str(tmp_path / "run"), max_restarts=2))
    t0 = time.time()
    while job.status not in ("succeeded", "failed", "nan_halt") and time.time() - t0 < 400:
        time.sleep(0.2)
    log = open(job.log_path).read()
    assert job.status == "succeeded", log[-4000:]
    assert job.restarts == 1 and job.world_history[-1] == 4, (job.restarts, job.world_history)
    assert "resumed from step 2" in log
    d = _dumps(tmp_path / "dump", 4)
    assert [x["rc"] for x in d] == [0] * 4 and all(x["step_count"] == 6 for x in d)
