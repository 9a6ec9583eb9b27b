"""Every REST endpoint of the reference through FastAPI's TestClient, plus the fixes."""
import os

import pytest
from fastapi.testclient import TestClient

os.environ["DLGM_TELEMETRY_INTERVAL_S"] = "0"
from backend.main import app  # noqa: E402

client = TestClient(app)


def test_root_and_health():
    r = client.get("/")
    assert r.status_code == 200 and r.json()["name"] == "MLOps Platform API" and len(r.json()["features"]) == 3
    assert client.get("/health").json() == {"status": "healthy"}


def test_gpu_endpoints_without_gpus():
    f = client.get("/api/v1/gpu/fleet").json()
    assert "devices" in f and "alerts" in f
    m = client.get("/api/v1/gpu/fleet/mock").json()
    assert m["total_gpus"] == 2 and m["devices"][0]["name"] == "AMD Instinct MI355X"
    s = client.get("/api/v1/gpu/select", params={"required_memory_mib": 1000})
    assert s.status_code == 200 and "recommendation" in s.json()
    assert client.get("/api/v1/gpu/select", params={"required_memory_mib": 10 ** 9}).status_code == 503
    assert client.get("/api/v1/gpu/devices/99").status_code == 404
    a = client.get("/api/v1/gpu/alerts").json()
    assert set(a) == {"total_alerts", "alerts", "devices_with_alerts"}


def test_topology_mounted():
    for path in ("/topology", "/api/v1/topology"):
        r = client.get(path)
        assert r.status_code == 200 and r.json()["interconnect"].startswith("xGMI")


def test_training_launch_dry_run_and_validation():
    r = client.post("/api/v1/training/launch", json={"training_script": "train.py", "model_name": "m", "bf16": True})
    assert r.status_code == 200
    j = r.json()
    assert j["status"] == "dry_run" and j["num_gpus"] == 1 and j["effective_batch_size"] == 32
    assert j["details"]["precision"] == "bf16"
    bad = client.post("/api/v1/training/launch", json={"training_script": "t.py", "offload_optimizer": "gpu"})
    assert bad.status_code == 422  # A16 (reference: 500)
    assert client.post("/api/v1/training/launch", json={"training_script": "t.py", "zero_stage": 4}).status_code == 422


def test_presets_and_preset_launch():
    p = client.get("/api/v1/training/presets").json()
    assert p["70b"]["num_nodes"] == 2 and p["70b"]["precision"] == "bf16" and p["7b"]["micro_batch_size"] == 2
    r = client.post("/api/v1/training/launch/preset", json={"preset": "13b", "training_script": "t.py"})
    assert r.status_code == 200 and r.json()["effective_batch_size"] == 256
    r = client.post("/api/v1/training/launch/preset", json={"preset": "nope", "training_script": "t.py"})
    assert r.status_code == 400 and "Available" in r.json()["detail"]


def test_config_generate_is_pure(tmp_path, monkeypatch):
    import tempfile

    # every tempfile-based write lands in tmp_path; /tmp itself is shared with concurrent test workers,
    # so only config-looking new names there count
    monkeypatch.setattr(tempfile, "tempdir", str(tmp_path))
    before = set(os.listdir("/tmp"))
    r = client.post("/api/v1/training/config/generate", json={"training_script": "t.py", "num_gpus": 8})
    assert r.status_code == 200
    j = r.json()
    assert j["deepspeed_config"]["zero_optimization"]["stage"] == 3 and j["effective_batch_size"] == 256
    assert "--nproc-per-node=8" in j["launch_command"]
    assert os.listdir(tmp_path) == []  # A24: no temp file written
    new = set(os.listdir("/tmp")) - before
    assert not [n for n in new if "ds_config" in n or "deepspeed" in n], new


def test_monitoring_flow_and_nan_safety():
    jid = "api-job"
    r = client.post("/api/v1/monitoring/create", json={"job_id": jid, "window_size": 50})
    assert r.json()["status"] == "created" and r.json()["config"]["window_size"] == 50
    r = client.post("/api/v1/monitoring/create", json={"job_id": jid, "window_size": 10})
    assert r.json()["status"] == "exists" and r.json()["config"]["window_size"] == 50  # A15
    assert client.get(f"/api/v1/monitoring/summary/{jid}").status_code == 200  # A14: inf best_loss
    metrics = [{"step": i, "loss": 2.0 + (3.0 if i == 30 else 0.0)} for i in range(40)]
    r = client.post("/api/v1/monitoring/ingest", json={"job_id": jid, "metrics": metrics}).json()
    assert r["ingested"] == 40 and any(a["alert_type"] == "spike" for a in r["alerts"])
    body = '{"job_id": "%s", "step": 41, "loss": NaN}' % jid  # what a Python client's json.dumps sends
    r = client.post("/api/v1/monitoring/ingest/single", content=body, headers={"content-type": "application/json"})
    assert r.status_code == 200 and r.json()["healthy"] is False  # A14: reference returned 500
    assert r.json()["alerts"][0]["metric_value"] == "NaN"
    c = client.get(f"/api/v1/monitoring/loss-curve/{jid}").json()
    assert c["steps"][-1] == 41 and 30 in c["spike_steps"]
    jobs = client.get("/api/v1/monitoring/jobs").json()
    assert jobs["active_jobs"] >= 1
    assert client.delete(f"/api/v1/monitoring/reset/{jid}").json()["status"] == "reset"
    for path in ("summary", "loss-curve"):
        assert client.get(f"/api/v1/monitoring/{path}/missing").status_code == 404
    assert client.delete("/api/v1/monitoring/reset/missing").status_code == 404


def test_jobs_endpoints():
    assert client.get("/api/v1/training/jobs").json()["total_jobs"] >= 0
    assert client.get("/api/v1/training/jobs/none").status_code == 404
    assert client.post("/api/v1/training/jobs/none/cancel").status_code == 404
    assert client.post("/api/v1/training/jobs/none/preempt").status_code == 404


def test_prometheus_metrics_endpoint():
    from fastapi.testclient import TestClient

    from backend.main import app

    c = TestClient(app)
    r = c.post("/api/v1/monitoring/ingest/single", json={"job_id": "prom-job", "step": 3, "loss": 2.5,
                                                          "learning_rate": 1e-4, "gradient_norm": 0.7})
    assert r.status_code == 200
    r = c.get("/metrics")
    assert r.status_code == 200
    body = r.text
    assert 'dlgm_train_loss{job="prom-job"} 2.5' in body
    assert 'dlgm_train_step{job="prom-job"} 3.0' in body
