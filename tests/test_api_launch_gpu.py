"""SURVEY.md §7.4's minimum slice ON THE MI355X through the control plane: POST
/api/v1/training/launch (dry_run false) starts a supervised llama-tiny job on the GPU (the reference's entry point,
/root/reference/backend/routers/training.py:55-79); the trainer pushes its metrics to /api/v1/monitoring
(routers/monitoring.py:66-79); /api/v1/training/jobs/{id} reaches `succeeded`; /api/v1/gpu/fleet (amdsmi,
routers/gpu.py:12-19) shows the device with the job's HBM in use while it runs."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.gpu
def test_api_launch_trains_on_the_gpu_and_the_fleet_shows_it(monkeypatch):
    import api_launch

    monkeypatch.setenv("DLGM_TELEMETRY_INTERVAL_S", "0")
    with api_launch.Server() as srv:
        rec = api_launch.run("llama-tiny", srv.url, poll_s=0.25)
    job, fleet, summ = rec["job"], rec["fleet"], rec["monitoring_summary"]
    assert job["status"] == "succeeded", (job, rec["log_tail"][-2000:])
    assert summ.get("total_steps") == 300 and summ.get("best_loss") is not None, summ
    before, peak = fleet["before"], fleet["peak_during"]
    assert before["gfx_arch"] in ("gfx950", None) and "MI35" in (before["name"] or ""), before
    assert peak is not None, fleet
    # the job's context and caching allocator on the device, seen by amdsmi while it trained: at least 256 MiB more
    # HBM in use than before the launch (the rank is a child of the job's torchrun pid, so pids are not compared)
    grew = (peak["memory_used_mib"] or 0) - (before["memory_used_mib"] or 0)
    assert grew >= 256, (peak, before)
    assert "peak_allocated_GiB" in rec["log_tail"], rec["log_tail"][-2000:]  # the trainer's device-memory line
