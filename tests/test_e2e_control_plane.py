"""Minimum end-to-end slice through the control plane: POST /api/v1/training/launch
(non-dry-run) starts a supervised training job on the in-house engine; the trainer pushes its
metrics to /api/v1/monitoring over HTTP; the job and its loss summary are visible through the API."""
import os
import socket
import threading
import time

import httpx
import pytest
import uvicorn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture()
def server():
    os.environ["DLGM_TELEMETRY_INTERVAL_S"] = "0"
    from backend.main import app

    port = _port()
    srv = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="warning"))
    th = threading.Thread(target=srv.run, daemon=True)
    th.start()
    url = f"http://127.0.0.1:{port}"
    for _ in range(100):
        try:
            httpx.get(url + "/health", timeout=1)
            break
        except httpx.HTTPError:
            time.sleep(0.1)
    yield url
    srv.should_exit = True
    th.join(10)


def test_launch_train_and_monitor_over_http(server):
    script = os.path.join(ROOT, "distributed_llm_training_gpu_manager_amd", "train.py")
    r = httpx.post(server + "/api/v1/training/launch", json={
        "training_script": script, "model_name": "llama-tiny", "zero_stage": 2, "micro_batch_size": 2,
        "gradient_accumulation_steps": 2, "dry_run": False, "num_gpus": 1,
        "script_args": ["--model", "llama-tiny", "--seq-len", "64", "--steps", "3", "--device", "cpu",
                        "--metrics-url", server]}, timeout=30)
    assert r.status_code == 200, r.text
    res = r.json()
    assert res["status"] == "launched", res
    job_id = res["job_id"]
    t0 = time.time()
    job = {}
    while time.time() - t0 < 240:
        job = httpx.get(f"{server}/api/v1/training/jobs/{job_id}", timeout=5).json()
        if job.get("status") in ("succeeded", "failed"):
            break
        time.sleep(0.5)
    assert job.get("status") == "succeeded", job
    # the DeepSpeed JSON the API generated (offload_optimizer=cpu by default) ran on the ZeRO-Offload path
    log = open(job["log_path"]).read()
    assert "step" in log
    for _ in range(50):  # metrics are pushed asynchronously
        s = httpx.get(f"{server}/api/v1/monitoring/summary/{job_id}", timeout=5)
        if s.status_code == 200 and s.json().get("total_steps", 0) >= 3:
            break
        time.sleep(0.2)
    assert s.status_code == 200, s.text
    assert s.json()["total_steps"] == 3
    m = httpx.get(server + "/metrics", timeout=5).text
    assert f'dlgm_train_step{{job="{job_id}"}} 3.0' in m
