"""Checkpoint / resume / NaN-trap / spot / auto-resume drills on CPU (BASELINE configs 3-5 plumbing)."""
import json
import os
import signal
import sys
import threading
import time
from http.server import BaseHTTPRequestHandler, HTTPServer

import pytest
import torch

from distributed_llm_training_gpu_manager_amd.ckpt.checkpoint import AsyncCheckpointer, complete_tags
from distributed_llm_training_gpu_manager_amd.ckpt.spot import SpotInstanceResiliencyManager
from distributed_llm_training_gpu_manager_amd.engine.trainer import Trainer, parse_args
from distributed_llm_training_gpu_manager_amd.launcher.supervisor import (EXIT_NAN_HALT, EXIT_PREEMPTED,
                                                                         JobRegistry, JobSpec)
from distributed_llm_training_gpu_manager_amd.models import get_config
from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _train(tmp, *extra):
    return Trainer(parse_args(["--seq-len", "32", "--save-dir", str(tmp), "--log-interval", "100", *extra]))


def _master(tr):
    return tr.engine.master.clone()


def test_resume_is_bit_exact(tmp_path):
    a = _train(tmp_path / "a", "--steps", "6")
    assert a.run() == 0
    ref = _master(a)
    b = _train(tmp_path / "b", "--steps", "4", "--save-interval", "2")
    assert b.run() == 0
    c = _train(tmp_path / "b", "--steps", "6", "--resume", "auto")
    assert c.run() == 0
    assert c.engine.step_count == 6 and torch.equal(_master(c), ref)


def test_corrupt_latest_rolls_back(tmp_path):
    b = _train(tmp_path, "--steps", "4", "--save-interval", "2")
    b.run()
    assert complete_tags(str(tmp_path)) == ["global_step2", "global_step4"]
    f = tmp_path / "global_step4" / "zero_pp_rank_0_mp_rank_00_optim_states.pt"
    man = json.load(open(tmp_path / "global_step4" / "manifest_r0.json"))
    off = man["files"]["zero_pp_rank_0_mp_rank_00_optim_states.pt"]["master"]["offset"]
    data = bytearray(f.read_bytes())
    data[off + 100] ^= 0xFF
    f.write_bytes(bytes(data))
    c = _train(tmp_path, "--steps", "4")
    cs = c.ckpt.load("auto")
    assert cs["step"] == 2 and c.engine.step_count == 2 and "checksum" in c.ckpt.rollbacks[0]


def _fp16_engine(seed=0):
    mc = get_config("llama-tiny")
    ec = EngineConfig(zero_stage=3, micro_batch_size=2, seq_len=32, grad_accum=1, lr=3e-3, scheduler="constant",
                      init_device="cpu", fp16=True, initial_scale_power=24, hysteresis=2, loss_scale_window=1000,
                      seed=seed)
    return ZeroEngine(mc, ec, torch.device("cpu")), mc


def test_fp16_loss_scaler_survives_checkpoint(tmp_path):
    """The dynamic loss scale and its hysteresis / good-step counters are saved and restored (DeepSpeed keeps
    the scaler in the checkpoint): a resumed fp16 run does not restart at 2**initial_scale_power and
    overflow again (checkpoint.py:670)."""
    eng, mc = _fp16_engine()
    g = torch.Generator().manual_seed(0)
    for _ in range(6):
        t = torch.randint(0, mc.vocab_size, (2, 33), generator=g)
        eng.train_step([(t[:, :-1], t[:, 1:])])
    st = eng.scaler.state_dict()
    assert st["cur_scale"] < 2.0 ** 24  # backed off from the initial scale
    ck = AsyncCheckpointer(eng, str(tmp_path))
    ck.save(6, {"step": 6}, blocking=True)
    ck.close()
    e2, _ = _fp16_engine(seed=5)
    assert e2.scaler.scale == 2.0 ** 24
    ck2 = AsyncCheckpointer(e2, str(tmp_path))
    assert ck2.load("auto")["step"] == 6
    assert e2.scaler.state_dict() == st
    assert torch.equal(e2.scaler.state, eng.scaler.state)
    ck2.close()


def test_partial_restore_without_fallback_raises(tmp_path):
    """A candidate that fails after overwriting part of the optimizer state, with no older candidate to
    replace it, must not leave the engine to train from step 0 on a mix of checkpoints."""
    from distributed_llm_training_gpu_manager_amd.ckpt.checkpoint import CorruptCheckpoint
    b = _train(tmp_path, "--steps", "2", "--save-interval", "2")
    b.run()
    f = tmp_path / "global_step2" / "zero_pp_rank_0_mp_rank_00_optim_states.pt"
    man = json.load(open(tmp_path / "global_step2" / "manifest_r0.json"))
    info = man["files"]["zero_pp_rank_0_mp_rank_00_optim_states.pt"]["exp_avg"]  # master is read before it
    data = bytearray(f.read_bytes())
    data[info["offset"] + 100] ^= 0xFF
    f.write_bytes(bytes(data))
    c = _train(tmp_path, "--steps", "2")
    with pytest.raises(CorruptCheckpoint, match="partial restore"):
        c.ckpt.load("auto")


def test_reshard_world_change(tmp_path):
    """Elastic restore: a W=1 ZeRO-3 checkpoint loaded into a different partition layout."""
    mc = get_config("llama-tiny")
    e1 = ZeroEngine(mc, EngineConfig(zero_stage=3, seq_len=32, init_device="cpu"), torch.device("cpu"))
    e1.master.normal_()
    ck = AsyncCheckpointer(e1, str(tmp_path))
    ck.save(3, {"step": 3}, blocking=True)
    e2 = ZeroEngine(mc, EngineConfig(zero_stage=3, seq_len=32, init_device="cpu", seed=99), torch.device("cpu"))
    # fake a different layout by loading through the reshard path explicitly
    ck2 = AsyncCheckpointer(e2, str(tmp_path))
    meta = torch.load(tmp_path / "global_step3" / "mp_rank_00_model_states.pt", weights_only=True)
    mans = {0: json.load(open(tmp_path / "global_step3" / "manifest_r0.json"))}
    ck2._reshard_from(str(tmp_path / "global_step3"), meta, mans, True)
    assert torch.equal(e1.master, e2.master)


def test_nan_injection_halts_with_code_3(tmp_path):
    t = _train(tmp_path, "--steps", "6", "--inject-nan-step", "3")
    before = None
    rc = t.run()
    assert rc == EXIT_NAN_HALT
    assert t.log[-1]["step"] == 3  # halted at the poisoned step: latency 0 steps after detection
    assert any(a.alert_type == "divergence" for a in t.monitor._all_alerts)
    assert t.trap.halted and t.trap.trip_step == 3


class _Meta(BaseHTTPRequestHandler):
    notice = False

    def do_PUT(self):
        self.send_response(200)
        self.end_headers()
        self.wfile.write(b"token")

    def do_GET(self):
        if self.path.endswith("instance-action") and _Meta.notice:
            self.send_response(200)
            self.end_headers()
            self.wfile.write(json.dumps({"action": "terminate", "time": "2026-10-15T00:00:00Z"}).encode())
        else:
            self.send_response(404)
            self.end_headers()

    def log_message(self, *a):
        pass


def test_spot_manager_against_fake_metadata_server():
    srv = HTTPServer(("127.0.0.1", 0), _Meta)
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    base = f"http://127.0.0.1:{srv.server_port}"
    got = []
    mgr = SpotInstanceResiliencyManager(check_interval_sec=0.05, provider="aws", on_preemption=got.append,
                                        urls={"aws_token": base + "/latest/api/token",
                                              "aws_action": base + "/latest/meta-data/spot/instance-action"})
    assert mgr.check_once() is None
    _Meta.notice = True
    import asyncio
    n = asyncio.run(mgr.monitor_preemption_notices(None))
    assert n["provider"] == "aws" and n["action"] == "terminate" and got
    srv.shutdown()
    m2 = SpotInstanceResiliencyManager(provider="gcp", urls={"gcp": base + "/nothing"})
    m2.simulate = True
    assert m2.check_once()["provider"] == "simulated"


def test_spot_preemption_drill_emergency_checkpoint_and_restore(tmp_path):
    t = _train(tmp_path, "--steps", "10", "--preempt-at-step", "4")
    assert t.run() == EXIT_PREEMPTED
    assert complete_tags(str(tmp_path))[-1] == "global_step4"
    r = _train(tmp_path, "--steps", "6", "--resume", "auto")
    assert r.run() == 0 and r.log[0]["step"] == 5


def test_spot_notice_when_ready_waits_for_the_prepared_snapshot(tmp_path, monkeypatch):
    """--preempt-when-ready (the warm spot drill): the notice goes out at the first step >= K at which the
    checkpointer reports its snapshot buffer prepared -- here the third step it is asked."""
    asked = []
    monkeypatch.setattr(AsyncCheckpointer, "prepared", property(lambda self: asked.append(1) or len(asked) >= 3))
    t = _train(tmp_path, "--steps", "10", "--preempt-at-step", "2", "--preempt-when-ready")
    assert t.run() == EXIT_PREEMPTED
    assert complete_tags(str(tmp_path))[-1] == "global_step4" and len(asked) == 3


def test_supervised_sigkill_auto_resume_mttr(tmp_path):
    """BASELINE config 4 plumbing: mid-run SIGKILL -> supervisor relaunch -> rollback -> MTTR recorded."""
    reg = JobRegistry()
    argv = [sys.executable, "-m", "distributed_llm_training_gpu_manager_amd.train", "--steps", "8",
            "--seq-len", "32", "--save-interval", "2", "--kill-at-step", "5", "--device", "cpu"]
    job = reg.submit(JobSpec(job_id="drill", argv=argv, env={"PYTHONPATH": ROOT}, save_dir=str(tmp_path / "ck"),
                             run_dir=str(tmp_path / "run")))
    t0 = time.time()
    while job.status not in ("succeeded", "failed") and time.time() - t0 < 120:
        time.sleep(0.1)
    log = open(job.log_path).read()
    assert job.status == "succeeded", log
    assert job.exit_codes[0] == -signal.SIGKILL and job.restarts == 1
    assert "resumed from step 4" in log
    assert len(job.mttr_s) == 1 and job.mttr_s[0] > 0


def test_wall_clock_breakdown_timers():
    import torch

    from distributed_llm_training_gpu_manager_amd.models import get_config
    from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine

    mc = get_config("llama-tiny")
    eng = ZeroEngine(mc, EngineConfig(zero_stage=2, micro_batch_size=1, seq_len=16, grad_accum=2, init_device="cpu",
                                      wall_clock_breakdown=True), torch.device("cpu"))
    t = torch.randint(0, mc.vocab_size, (1, 17))
    eng.train_step([(t[:, :-1], t[:, 1:])] * 2)
    s = eng.timers.summary()
    assert s["forward"]["count"] == 2 and s["backward+reduce"]["count"] == 2 and s["optimizer_step"]["count"] == 1
    assert all(v["total_ms"] > 0 for v in s.values())
    assert eng.timers.summary() == {}


def test_zero_to_fp32_offline_consolidation(tmp_path):
    """ckpt/zero_to_fp32.py rebuilds the full fp32 parameters from the shard files alone (no engine)."""
    from distributed_llm_training_gpu_manager_amd.ckpt import zero_to_fp32

    mc = get_config("llama-tiny")
    eng = ZeroEngine(mc, EngineConfig(zero_stage=3, seq_len=32, init_device="cpu"), torch.device("cpu"))
    eng.master.normal_()
    eng.exp_avg.uniform_()
    ck = AsyncCheckpointer(eng, str(tmp_path))
    ck.save(5, {"step": 5}, blocking=True)
    full = eng.full_params()
    got = zero_to_fp32.consolidate(str(tmp_path))
    assert set(got) == set(full)
    for k, v in full.items():
        assert torch.equal(got[k], v.float()), k
    m1 = zero_to_fp32.consolidate(str(tmp_path), "global_step5", state="exp_avg")
    assert all(torch.equal(m1[k], v) for k, v in eng._gather_flat(eng.exp_avg).items())
    out = tmp_path / "w.safetensors"
    assert zero_to_fp32.main([str(tmp_path), str(out), "--dtype", "bf16"]) == 0
    from safetensors.torch import load_file
    sd = load_file(str(out))
    assert all(torch.equal(sd[k], v.to(torch.bfloat16)) for k, v in full.items())


def test_checkpointer_reports_prepared_after_background_preparation(tmp_path):
    """AsyncCheckpointer.prepared (what --preempt-when-ready waits for): False before the snapshot buffer exists,
    True once the background preparation has reserved the whole /dev/shm file (no GPU: nothing to page-lock)."""
    mc = get_config("llama-tiny")
    eng = ZeroEngine(mc, EngineConfig(zero_stage=3, micro_batch_size=1, seq_len=32, grad_accum=1,
                                      scheduler="constant", init_device="cpu"), torch.device("cpu"))
    ck = AsyncCheckpointer(eng, str(tmp_path), shm=True, disk=False)
    assert ck.mode == "shm" and not ck.prepared
    ck.prepare_async()
    ck._prep.join()
    assert ck.prepared and ck._falloc_done == ck.snap_bytes
    ck.save(1, {"step": 1}, blocking=True)
    assert ck.prepared
    ck.close(discard_shm=True)


@pytest.mark.parametrize("via", ["supervisor", "registry"])
def test_supervisor_reserves_shm_snapshots_before_the_first_launch(tmp_path, via):
    """the supervisor (which outlives the ranks) reserves each rank's /dev/shm snapshot file before
    the first launch, sized by the planner from the training command; the checkpointer then finds every page reserved
    (prep_stats.pre_reserved: only mapping / page-locking left for an early spot notice), and a second reservation
    never touches a snapshot that is already there (it is the restore source of a relaunch)."""
    from distributed_llm_training_gpu_manager_amd.ckpt.checkpoint import reserve_snapshot_files, shm_snapshot_path
    from distributed_llm_training_gpu_manager_amd.launcher.supervisor import (Job, JobRegistry, JobSpec, Supervisor,
                                                                               planned_snapshot_bytes)
    save = str(tmp_path / "ck")
    cmd = [sys.executable, "-c", "pass", "--model", "llama-tiny", "--zero-stage", "3"]
    nb = planned_snapshot_bytes(cmd, 1)
    eng = ZeroEngine(get_config("llama-tiny"), EngineConfig(zero_stage=3, micro_batch_size=1, seq_len=16,
                                                            init_device="cpu"), torch.device("cpu"))
    assert 14 * eng.shard_total <= nb <= 14 * eng.shard_total + (64 << 20)
    spec = JobSpec(job_id="shm", argv=cmd, save_dir=save, run_dir=str(tmp_path / "run"), shm_reserve_bytes=nb)
    if via == "supervisor":
        job = Job(spec)
        sup = Supervisor(job)
        sup.start()
        sup.join(60)
    else:  # the API / drill path: JobRegistry.submit starts the first attempt itself, synchronously
        job = JobRegistry().submit(spec)
        t0 = time.time()
        while job.status not in ("succeeded", "failed", "preempted") and time.time() - t0 < 60:
            time.sleep(0.05)
    ev = [e for e in job.events if e["event"] == "shm_reserved"]
    path = shm_snapshot_path(save, 0)
    try:
        assert ev and ev[0]["bytes_added"] == nb and os.path.exists(path), job.events
        st = os.stat(path)
        assert st.st_blocks * 512 >= nb
        ck = AsyncCheckpointer(eng, save, shm=True, disk=False)
        assert ck.mode == "shm" and ck.shm_path == path
        ck._alloc_snapshot()
        assert ck.prep_stats.get("pre_reserved") and ck._falloc_done == ck.snap_bytes
        ck.save(1, {"step": 1}, blocking=True)
        before, size = open(path, "rb").read(4096), os.path.getsize(path)  # the checkpointer trimmed the slack
        again = reserve_snapshot_files(save, [0], nb)
        assert again["bytes_added"] == nb - size and open(path, "rb").read(4096) == before
        ck.close()
    finally:
        for p in (path, path[:-5] + ".json"):
            if os.path.exists(p):
                os.unlink(p)
