#!/usr/bin/env python3
"""Resilience drills on real hardware -> JSON (BASELINE configs 3-5 metrics).

  nan     : inject a NaN gradient at step K -> steps & ms until the job halts (exit 3)
  sigkill : supervised run, SIGKILL at step K -> auto-resume -> MTTR (failure detected -> first
            completed step after the restart), plus checkpoint capture / write / restore times
  spot    : SIGUSR1 at step K (what the spot manager sends) -> emergency checkpoint -> exit 4 ->
            restore on a fresh process -> first step
  spot_warm: the same with the notice at the first step >= K at which the snapshot buffer is prepared
"""
from __future__ import annotations

import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_llm_training_gpu_manager_amd.launcher.supervisor import JobRegistry, JobSpec  # noqa: E402


def train_argv(a, extra):
    return [sys.executable, "-m", "distributed_llm_training_gpu_manager_amd.train", "--model", a.model,
            "--seq-len", str(a.seq), "--micro-batch", "1", "--grad-accum", str(a.ga), "--zero-stage", "3",
            "--lr", "3e-5", *(["--n-layers", str(a.n_layers)] if a.n_layers else []),
            "--keep-last", str(a.keep_last), "--ckpt-shm", a.ckpt_shm, "--ckpt-disk", str(a.ckpt_disk),
            *a.extra.split(), *extra]


def run(argv, timeout):
    t0 = time.time()
    p = subprocess.run(argv, capture_output=True, text=True, timeout=timeout, cwd=ROOT,
                       env={**os.environ, "PYTHONPATH": ROOT})
    return p.returncode, p.stdout + p.stderr, time.time() - t0


def drill_nan(a, work):
    log = os.path.join(work, "nan.json")
    rc, out, dt = run(train_argv(a, ["--steps", str(a.k + 3), "--inject-nan-step", str(a.k), "--log-json", log]),
                      a.timeout)
    d = json.load(open(log)) if os.path.exists(log) else {}
    steps = [r["step"] for r in d.get("log", [])]
    trap = d.get("trap", [])
    return {"drill": "nan", "exit_code": rc, "inject_step": a.k, "last_step_run": steps[-1] if steps else None,
            "halt_latency_steps": (steps[-1] - a.k) if steps else None,
            "halt_latency_ms": None if not d.get("log") else round(1000 * d["log"][-1]["step_s"], 1),
            "trap_records": trap[-3:], "tail": out[-600:]}


def drill_sigkill(a, work):
    ck = os.path.join(work, "ck")
    reg = JobRegistry()
    argv = train_argv(a, ["--steps", str(a.k + 2 + a.steps_after), "--save-interval", str(a.save_interval), "--kill-at-step",
                          str(a.k), "--log-json", os.path.join(work, "kill.json")])
    t0 = time.time()
    job = reg.submit(JobSpec(job_id="sigkill-drill", argv=argv, env={"PYTHONPATH": ROOT}, save_dir=ck,
                             run_dir=os.path.join(work, "run")))
    while job.status not in ("succeeded", "failed") and time.time() - t0 < a.timeout:
        time.sleep(0.2)
    log = open(job.log_path).read()
    resumed = re.findall(r"resumed from step (\d+) in ([0-9.]+)s", log)
    via = re.findall(r"resumed from step \d+ in [0-9.]+s via (\S+)", log)
    stats = [json.loads(x) for x in re.findall(r"restore (\{.*?\})\)", log)]
    startup = [json.loads(x) for x in re.findall(r"\[train\] startup: (\{.*?\})", log)]
    hist, steps_after = {}, []
    if os.path.exists(os.path.join(work, "kill.json")):
        kj = json.load(open(os.path.join(work, "kill.json")))
        hist = kj.get("ckpt", [])
        steps_after = [[r["step"], round(r["step_s"], 2)] for r in kj.get("log", [])]
    return {"drill": "sigkill", "status": job.status, "exit_codes": job.exit_codes, "restarts": job.restarts,
            "mttr_s": [round(x, 2) for x in job.mttr_s], "resume_load_s": [float(s) for _, s in resumed],
            "resumed_from_step": [int(s) for s, _ in resumed], "restored_from": via, "restore_breakdown": stats,
            "startup_timeline": startup,  # per launch: imports / process group / engine / restore / first step
            "step_timing": re.findall(r"step-timing: (.*)", log),  # DLGM_STEP_TIMING: issue vs device-done per step
            "ckpt_prepare": [json.loads(x) for x in re.findall(r"ckpt prepare: (\{.*?\})", log)],
            "memory": [json.loads(x) for x in re.findall(r"memory: (\{.*?\})", log)],
            "events": job.events,
            "ckpt_after_resume": hist,
            "step_s_after_resume": steps_after,
            "tail": log[-800:]}


def drill_spot(a, work, warm=False):
    """warm: the notice lands once the snapshot buffer is prepared (--preempt-when-ready) instead of at step K."""
    ck = os.path.join(work, "ck_spot")
    notice = ["--preempt-at-step", str(a.k)] + (["--preempt-when-ready"] if warm else [])
    rc, out, dt = run(train_argv(a, ["--steps", str(a.k + (400 if warm else 5)), "--save-dir", ck, *notice]),
                      a.timeout)
    em = re.findall(r"emergency checkpoint at step (\d+) in ([0-9.]+)s", out)
    rc2, out2, dt2 = run(train_argv(a, ["--steps", str(a.k + 1), "--save-dir", ck, "--resume", "auto"]), a.timeout)
    res = re.findall(r"resumed from step (\d+) in ([0-9.]+)s", out2)
    via = re.findall(r"resumed from step \d+ in [0-9.]+s via (\S+)", out2)
    stats = re.findall(r"restore (\{.*?\})\)", out2)
    return {"drill": "spot_warm" if warm else "spot", "restore_breakdown": [json.loads(x) for x in stats], "exit_code_preempted": rc,
            "emergency_ckpt": em, "restore_exit": rc2,
            "emergency_record": [json.loads(x) for x in re.findall(r"emergency checkpoint record: (\{.*?\})\n", out)],
            "memory": [json.loads(x) for x in re.findall(r"memory: (\{.*?\})", out + out2)],
            "ckpt_prepare": [json.loads(x) for x in re.findall(r"ckpt prepare: (\{.*?\})", out + out2)],
            "restore": res, "restored_from": via, "restore_process_wall_s": round(dt2, 2),
            "tail": (out[-300:], out2[-300:])}


def drill_spot_reserved(a, work):
    """spot_reserved: the job runs under the supervisor, which reserves this rank's /dev/shm
    snapshot file (planner size from the command) BEFORE the first launch; the spot notice lands at step 1 -- before
    the trainer's own background preparation could have prepared a fresh file -- and the emergency checkpoint must
    finish inside the 120 s notice window (/root/reference/ai_engine/spot_resiliency.py:8-10) with a wide margin.
    Then a fresh process restores from it."""
    from distributed_llm_training_gpu_manager_amd.launcher.supervisor import planned_snapshot_bytes
    ck = os.path.join(work, "ck_spot_res")
    argv = train_argv(a, ["--steps", "6", "--save-dir", ck, "--preempt-at-step", "1"])
    nb = planned_snapshot_bytes(argv, 1)
    t0 = time.time()
    job = JobRegistry().submit(JobSpec(job_id="spot-reserved-drill", argv=argv, env={"PYTHONPATH": ROOT}, save_dir=ck,
                                       run_dir=os.path.join(work, "run_spot_res"), auto_resume=False,
                                       shm_reserve_bytes=nb))
    while job.status not in ("succeeded", "failed", "preempted") and time.time() - t0 < a.timeout:
        time.sleep(0.2)
    log = open(job.log_path).read()
    em = re.findall(r"emergency checkpoint at step (\d+) in ([0-9.]+)s", log)
    rc2, out2, dt2 = run(train_argv(a, ["--steps", "2", "--save-dir", ck, "--resume", "auto"]), a.timeout)
    res = re.findall(r"resumed from step (\d+) in ([0-9.]+)s", out2)
    ck_s = float(em[0][1]) if em else None
    return {"drill": "spot_reserved", "status": job.status, "exit_codes": job.exit_codes,
            "shm_reserved": [e for e in job.events if e["event"] == "shm_reserved"],
            "planned_snapshot_bytes": nb, "emergency_ckpt": em,
            "notice_window_s": 120.0, "margin_to_notice_window_s": None if ck_s is None else round(120.0 - ck_s, 2),
            "emergency_record": [json.loads(x) for x in re.findall(r"emergency checkpoint record: (\{.*?\})\n", log)],
            "ckpt_prepare": [json.loads(x) for x in re.findall(r"ckpt prepare: (\{.*?\})", log + out2)],
            "startup_timeline": [json.loads(x) for x in re.findall(r"\[train\] startup: (\{.*?\})", log)],
            "restore_exit": rc2, "restore": res, "restore_process_wall_s": round(dt2, 2),
            "events": job.events, "tail": (log[-600:], out2[-300:])}


def _drop_shm(save_dir: str) -> None:
    """Remove the /dev/shm snapshot tier a drill's save dir left behind (failed runs keep it for resume)."""
    import glob
    import hashlib
    key = hashlib.sha1(os.path.abspath(save_dir).encode()).hexdigest()[:12]
    for p in glob.glob(f"/dev/shm/dlgm-ckpt-{key}-*"):
        try:
            os.unlink(p)
        except OSError:
            pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--drills", default="nan,sigkill,spot")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--n-layers", type=int, default=0)
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--ga", type=int, default=1)
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--save-interval", type=int, default=2)
    ap.add_argument("--steps-after", type=int, default=0, help="sigkill drill: extra steps after the resume")
    ap.add_argument("--timeout", type=float, default=900)
    ap.add_argument("--keep-last", type=int, default=1)
    ap.add_argument("--ckpt-shm", default="auto", choices=["auto", "on", "off"])
    ap.add_argument("--ckpt-disk", type=int, default=1, help="0: /dev/shm snapshot tier only (no disk tags)")
    ap.add_argument("--extra", default="", help="more trainer arguments, e.g. '--shadow-world 8 --shadow-rank 0' "
                    "(rank 0 of an 8-rank job alone on this GPU: the 70B config-4 drill at true per-rank size)")
    ap.add_argument("--out", default="gpurun_out/drills.json")
    ap.add_argument("--work", default=None)
    a = ap.parse_args()
    work = a.work or tempfile.mkdtemp(prefix="dlgm_drill_")
    res = {"model": a.model, "n_layers": a.n_layers or "preset", "seq": a.seq, "ga": a.ga, "extra": a.extra,
           "keep_last": a.keep_last, "ckpt_shm": a.ckpt_shm, "ckpt_disk": a.ckpt_disk,
           "data": "synthetic token ids, random-init weights"}
    for d in a.drills.split(","):
        t0 = time.time()
        res[d] = {"nan": drill_nan, "sigkill": drill_sigkill, "spot": drill_spot, "spot_reserved": drill_spot_reserved,
                  "spot_warm": lambda a_, w_: drill_spot(a_, w_, warm=True)}[d](a, work)
        res[d]["wall_s"] = round(time.time() - t0, 1)
        print(json.dumps({k: v for k, v in res[d].items() if k != "tail"})[:2000], flush=True)
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
        for sub in ("ck", "ck_spot", "ck_spot_res"):  # the box's scratch disk holds one drill's checkpoints at a time
            shutil.rmtree(os.path.join(work, sub), ignore_errors=True)
            _drop_shm(os.path.join(work, sub))
    shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
