"""MI355X runtime paths around the kernels: live amdsmi telemetry, the /dev/shm checkpoint tier with a
page-locked (hipHostRegister) snapshot, and the trainer's one-step-late host loop with the NaN latch."""
import os
import time

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_live_amdsmi_query_and_topology():
    from distributed_llm_training_gpu_manager_amd.health.gpu_manager import GPUManager

    mgr = GPUManager()
    devs = mgr.query_amdsmi()
    assert devs, "amdsmi sees no GPU"
    d = devs[0]
    assert d.memory_total_mib > 200 * 1024, d.memory_total_mib  # 288 GB HBM3E
    assert (d.hotspot_temperature_celsius or d.temperature_celsius) > 0
    assert d.power_limit_watts > 0
    topo = mgr.topology()
    assert topo["source"] in ("amdsmi", "none") and "topology_matrix" in topo
    fleet = mgr.get_fleet_status()
    assert fleet.total_gpus >= 1 and fleet.source in ("amdsmi", "amd-smi-cli")


def test_in_job_telemetry_sampler():
    from distributed_llm_training_gpu_manager_amd.health.telemetry import TelemetrySampler

    s = TelemetrySampler(torch.device("cuda", 0), interval_s=0.2).start()
    x = torch.randn(8192, 8192, device="cuda")
    for _ in range(20):
        x = x @ x.t()
        x = x / x.norm()
    torch.cuda.synchronize()
    time.sleep(0.5)
    out = s.stop()
    assert out["samples"] >= 2 and out["source"] == "amdsmi", out
    assert out["junction_temp_c"]["max"] > 0 and out["hbm_used_gib"]["max"] > 0
    assert "Radeon" not in out["device"] and "MI35" in out["device"], out["device"]  # the product, not libdrm's default
    assert all(isinstance(a, dict) and a["count"] >= 1 for a in out.get("alerts", []))


def _engine(seed=0):
    from distributed_llm_training_gpu_manager_amd.models import get_config
    from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine

    return ZeroEngine(get_config("llama-small"), EngineConfig(zero_stage=3, seq_len=256, micro_batch_size=1,
                                                              grad_accum=1, seed=seed, scheduler="constant"),
                      torch.device("cuda", 0))


def test_shm_tier_checkpoint_roundtrip(tmp_path):
    from distributed_llm_training_gpu_manager_amd.ckpt.checkpoint import AsyncCheckpointer

    e = _engine()
    t = torch.randint(0, 32768, (1, 257), device="cuda")
    e.train_step([(t[:, :-1], t[:, 1:])])
    ck = AsyncCheckpointer(e, str(tmp_path), shm=True)
    assert ck.mode == "shm"
    ck.save(1, {"step": 1}, blocking=True)
    assert ck._pinned_shm, "hipHostRegister of the /dev/shm snapshot failed"
    want = e.master.clone()
    e.train_step([(t[:, :-1], t[:, 1:])])  # the optimizer waits for the capture on the GPU
    ck.close()
    e2 = _engine(seed=3)
    ck2 = AsyncCheckpointer(e2, str(tmp_path), shm=True)
    assert ck2.load("auto")["step"] == 1 and ck2.restored_from == "shm:global_step1"
    assert torch.equal(e2.master, want)
    ck2.close(discard_shm=True)
    d = torch.load(tmp_path / "global_step1" / "zero_pp_rank_0_mp_rank_00_optim_states.pt", weights_only=True)
    assert torch.equal(d["optimizer_state_dict"]["fp32_flat_groups"][0], want.cpu())


def test_shm_restore_defers_moments_behind_the_first_step(tmp_path):
    """The shm restore returns once the master is on the device; the Adam moments follow on a background
    thread while the next step's forward / backward runs, and that step's optimizer waits for them. The
    trained state must equal a restore that copied everything before returning."""
    from distributed_llm_training_gpu_manager_amd.ckpt.checkpoint import AsyncCheckpointer

    e = _engine()
    t = torch.randint(0, 32768, (1, 257), device="cuda")
    for _ in range(2):
        e.train_step([(t[:, :-1], t[:, 1:])])
    ck = AsyncCheckpointer(e, str(tmp_path), shm=True, disk=False)
    ck.save(2, {"step": 2}, blocking=True)
    ck.close()
    out = {}
    for defer in (False, True):
        e2 = _engine(seed=5)
        ck2 = AsyncCheckpointer(e2, str(tmp_path), shm=True, disk=False)
        ck2.defer_moments = defer
        assert ck2.load("auto")["step"] == 2 and ck2.restored_from == "shm:global_step2"
        assert ("deferred_GiB" in ck2.restore_stats) == defer, ck2.restore_stats
        e2.train_step([(t[:, :-1], t[:, 1:])])  # the optimizer joins the deferred copies
        assert ck2._moments is None
        out[defer] = [x.clone() for x in (e2.master, e2.exp_avg, e2.exp_avg_sq)]
        ck2.close()
        del e2, ck2
    for a, b in zip(out[False], out[True]):
        assert torch.equal(a, b)
    AsyncCheckpointer(_engine(), str(tmp_path), shm=True, disk=False).close(discard_shm=True)


@pytest.mark.gpu
def test_shm_save_falls_back_to_host_when_the_reservation_fails(tmp_path, monkeypatch):
    """an early save reserves the rest of the shm file itself; when the tmpfs fills up there (a failed
    posix_fallocate), the save must not crash and lose the emergency checkpoint: it drops the shm file and captures
    the state into a pinned host buffer instead."""
    from distributed_llm_training_gpu_manager_amd.ckpt import checkpoint as C

    monkeypatch.setattr(C, "REG_CHUNK", 64 << 20)
    monkeypatch.setattr(C, "REG_PAUSE_S", 0.05)
    e = _engine()
    t = torch.randint(0, 32768, (1, 257), device="cuda")
    e.train_step([(t[:, :-1], t[:, 1:])])
    ck = C.AsyncCheckpointer(e, str(tmp_path), shm=True, disk=False)
    assert ck.mode == "shm" and ck.snap_bytes > 4 * (64 << 20)
    real, calls = ck._reserve, []

    def slow_then_full(fd, off, ln):
        # the background preparation reserves slowly (a tmpfs reserves ~17 GB/s: unthrottled, the whole file would be
        # reserved before the save arrives); the save's own reservation of the rest finds the tmpfs full. (The save
        # joins the preparation thread and clears ck._prep before it reserves anything itself.)
        calls.append((off, ck._prep is not None))
        if ck._prep is None:
            ck.tier_notes.append("No space left on device (simulated)")
            return False
        time.sleep(0.03)
        return real(fd, off, ln)
    monkeypatch.setattr(ck, "_reserve", slow_then_full)
    ck.prepare_async()
    time.sleep(0.12)  # a few pieces prepared, most not
    ck.save(1, {"step": 1}, blocking=True)
    assert any(not prep for _, prep in calls), calls  # the save itself hit the full tmpfs
    rec = ck.history[-1]
    assert ck.mode == "host" and rec["mode"] == "host", rec
    assert any("snapshot tier -> host memory" in n for n in ck.tier_notes), ck.tier_notes
    assert not os.path.exists(ck.shm_path) and not os.path.exists(ck.shm_meta)
    assert torch.equal(ck._snap[:4 * ck.n].view(torch.float32), e.master.cpu())
    e.train_step([(t[:, :-1], t[:, 1:])])
    ck.save(2, {"step": 2}, blocking=True)  # later saves keep working on the host tier
    assert torch.equal(ck._snap[:4 * ck.n].view(torch.float32), e.master.cpu())
    ck.close()



@pytest.mark.parametrize("register_fails", [False, True])
def test_shm_save_before_preparation_finishes(tmp_path, monkeypatch, register_fails):
    """An early save (a spot notice in the first steps) interrupts the background reservation / page-locking: the
    page-locked prefix goes by DMA and the save page-locks the rest itself, piece by piece, each piece's DMA queued
    as soon as it is locked; when page-locking fails, the rest goes through the pinned slots with on-the-fly CRCs.
    The snapshot holds the state (CRCs agree with a full recomputation), a later save works, and it restores."""
    from distributed_llm_training_gpu_manager_amd.ckpt import checkpoint as C

    monkeypatch.setattr(C, "REG_CHUNK", 64 << 20)
    monkeypatch.setattr(C, "REG_PAUSE_S", 0.05)
    e = _engine()
    t = torch.randint(0, 32768, (1, 257), device="cuda")
    e.train_step([(t[:, :-1], t[:, 1:])])
    ck = C.AsyncCheckpointer(e, str(tmp_path), shm=True, disk=False)
    assert ck.mode == "shm" and ck.snap_bytes > 4 * (64 << 20)
    ck.prepare_async()
    time.sleep(0.12)  # a few pieces prepared, most not
    if register_fails:  # what is not page-locked yet can no longer be
        fns = ck._hip_register_fns()
        monkeypatch.setattr(ck, "_hip_register_fns", lambda: ((lambda p_, n_: 1), fns[1]))
    ck.save(1, {"step": 1}, blocking=True)
    rec = ck.history[-1]
    assert "ring" in rec, rec
    if register_fails:
        assert 0 < rec["ring"]["bytes"] < ck.snap_bytes and rec["ring"]["locked_bytes"] == 0, rec
    else:
        assert rec["ring"]["locked_bytes"] > 0 and "bytes" not in rec["ring"] and ck._pinned_shm, rec
    want = e.master.clone()
    import json

    from distributed_llm_training_gpu_manager_amd import _host
    with open(ck.shm_meta) as f:
        meta = json.load(f)
    snap = torch.from_file(ck.shm_path, shared=False, size=ck.snap_bytes, dtype=torch.uint8)
    assert _host.crc32c_chunks(snap) == meta["crc"]
    assert torch.equal(snap[:4 * ck.n].view(torch.float32), want.cpu())
    del snap
    if ck._prep is not None:
        ck._prep.join()
    e.train_step([(t[:, :-1], t[:, 1:])])
    ck.save(2, {"step": 2}, blocking=True)
    want2 = e.master.clone()
    ck.close()
    e2 = _engine(seed=3)
    ck2 = C.AsyncCheckpointer(e2, str(tmp_path), shm=True, disk=False)
    assert ck2.load("auto")["step"] == 2
    assert torch.equal(e2.master, want2) and not torch.equal(want, want2)
    ck2.close(discard_shm=True)


def _trainer(tmp, *extra):
    from distributed_llm_training_gpu_manager_amd.engine.trainer import Trainer, parse_args

    return Trainer(parse_args(["--model", "llama-small", "--seq-len", "2048", "--device", "cuda",
                               "--log-interval", "100", "--telemetry-interval", "0", *extra]))


@pytest.mark.no_stream_audit  # asserts host run-ahead: the audit's per-op Python work lets the GPU catch up
def test_trainer_runs_ahead_and_nan_latch_keeps_pre_nan_state(tmp_path):
    from distributed_llm_training_gpu_manager_amd.launcher.supervisor import EXIT_NAN_HALT

    ok = _trainer(tmp_path, "--steps", "8")
    assert ok.run() == 0
    # every report but the last was read with the next step already queued (the host never drains the GPU
    # to decide), and at least some of those reads found their step still running on the device
    assert ok.read_behind == 7, ok.read_behind
    assert ok.trap.waited >= 1, ok.trap.waited
    ref = _trainer(tmp_path, "--steps", "2")
    assert ref.run() == 0
    bad = _trainer(tmp_path, "--steps", "8", "--inject-nan-step", "3")
    assert bad.run() == EXIT_NAN_HALT
    assert bad.trap.trip_step == 3 and bad.log[-1]["step"] == 3
    # step 4 was queued before the halt decision; the device latch skipped its update too
    assert bad.engine.step_count >= 4
    assert torch.equal(bad.engine.master, ref.engine.master)


def test_offload_param_on_gpu_matches_device_params(tmp_path):
    """offload_param=cpu: the bf16 partition in pinned host memory, H2D-staged gathers on a side stream;
    offload_param=nvme: the partition in a file, read per gather by the C++ AIO engine into pinned ring slots
    (released by the H2D copy's event) and written back after each device AdamW step."""
    from distributed_llm_training_gpu_manager_amd.models import get_config
    from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine

    res = {}
    for name, off in (("dev", "none"), ("host", "cpu"), ("nvme", "nvme")):
        torch.cuda.empty_cache()
        e = ZeroEngine(get_config("llama-small"), EngineConfig(zero_stage=3, seq_len=512, micro_batch_size=1,
                                                               grad_accum=2, scheduler="constant", offload_param=off,
                                                               nvme_path=str(tmp_path / "nvme")),
                       torch.device("cuda", 0))
        g = torch.Generator(device="cuda").manual_seed(0)
        for _ in range(2):
            mb = [torch.randint(0, 32768, (1, 513), device="cuda", generator=g) for _ in range(2)]
            m = e.train_step([(t[:, :-1], t[:, 1:]) for t in mb])
        torch.cuda.synchronize()
        res[name] = (float(m["loss"]), e.master.clone(), e.p16_shard.device.type, e.memory_report(),
                     dict(e.param_nvme.stats) if e.param_nvme is not None else None)
        del e
    assert res["host"][2] == "cpu" and res["dev"][2] == "cuda"
    assert res["host"][3]["param_shard_host_GiB"] > 0 and res["host"][3]["param_shard_GiB"] == 0
    st = res["nvme"][4]
    assert st is not None and st["read_GiB"] > 0 and st["write_GiB"] > 0, st
    for name in ("host", "nvme"):
        assert abs(res[name][0] - res["dev"][0]) < 1e-3, name
        assert torch.equal(res[name][1], res["dev"][1]), name
