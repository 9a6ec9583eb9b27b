#!/usr/bin/env python3
"""SURVEY.md §7.4's minimum slice on the MI355X, through the control plane.

The reference's entry point is ``POST /api/v1/training/launch`` (``/root/reference/backend/routers/training.py:55-79``
-> ``deepspeed_launcher.py:302-367``); metrics reach ``/api/v1/monitoring`` (``routers/monitoring.py:66-79``) and the
fleet is visible at ``/api/v1/gpu/fleet`` (``routers/gpu.py:12-19``). This driver starts the FastAPI app in-process
(uvicorn on 127.0.0.1), launches a NON-dry-run job through the API, polls ``/api/v1/training/jobs/{id}`` and
``/api/v1/gpu/fleet`` (amdsmi) while it runs, and returns the job's events, its monitoring summary and the fleet
snapshots (before, during -- the one with the most HBM in use -- and after).

    python tools/api_launch.py --preset llama3-8b --out profiles/api_launch_llama3_8b_r06.json

``tests/test_api_launch_gpu.py`` drives the same function with llama-tiny.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import threading
import time
from typing import Any, Dict, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

PRESETS = {
    # BASELINE config 2: Llama-3-8B ZeRO-3 bf16, seq 8192, mbs 1 x GA 8 (the headline), 5 optimizer steps
    "llama3-8b": dict(request=dict(model_name="llama3-8b", zero_stage=3, micro_batch_size=1,
                                   gradient_accumulation_steps=8, fp16=False, bf16=True, offload_optimizer="none",
                                   offload_param="none", activation_checkpointing=False, learning_rate=3e-5),
                      args=["--model", "llama3-8b", "--seq-len", "8192", "--steps", "5"], timeout_s=900),
    "llama-tiny": dict(request=dict(model_name="llama-tiny", zero_stage=3, micro_batch_size=4,
                                    gradient_accumulation_steps=2, fp16=False, bf16=True, offload_optimizer="none",
                                    offload_param="none", activation_checkpointing=False, learning_rate=1e-3),
                       args=["--model", "llama-tiny", "--seq-len", "512", "--steps", "300"], timeout_s=300),
}


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Server:
    """The control plane's FastAPI app on a uvicorn thread (127.0.0.1, a free port)."""

    def __init__(self):
        import uvicorn
        from backend.main import app
        self.port = _port()
        self.srv = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=self.port, log_level="warning"))
        self.th = threading.Thread(target=self.srv.run, daemon=True)
        self.url = f"http://127.0.0.1:{self.port}"

    def __enter__(self):
        import httpx
        self.th.start()
        for _ in range(200):
            try:
                httpx.get(self.url + "/health", timeout=1)
                break
            except httpx.HTTPError:
                time.sleep(0.1)
        return self

    def __exit__(self, *exc):
        self.srv.should_exit = True
        self.th.join(10)
        return False


def _fleet_dev(fleet: Dict[str, Any], t0: float) -> Dict[str, Any]:
    d = (fleet.get("devices") or [{}])[0]
    return {"t_s": round(time.time() - t0, 2), "name": d.get("name"), "gfx_arch": d.get("gfx_arch"),
            "memory_used_mib": d.get("memory_used_mib"), "memory_total_mib": d.get("memory_total_mib"),
            "gpu_utilization_pct": d.get("gpu_utilization_pct"), "power_draw_watts": d.get("power_draw_watts"),
            "temperature_celsius": d.get("temperature_celsius"),
            "hbm_temperature_celsius": d.get("hbm_temperature_celsius"), "health": d.get("health"),
            "processes": [{"pid": p.get("pid"), "used_memory_mib": p.get("used_memory_mib")}
                          for p in d.get("processes") or []],
            "fleet_alerts": fleet.get("alerts", [])[:4]}


def run(preset: str, url: str, extra_args: Optional[List[str]] = None, poll_s: float = 1.0) -> Dict[str, Any]:
    """Launch `preset` through POST /api/v1/training/launch on the server at `url` and follow it to the end."""
    import httpx
    p = PRESETS[preset]
    script = os.path.join(ROOT, "distributed_llm_training_gpu_manager_amd", "train.py")
    t0 = time.time()
    before = _fleet_dev(httpx.get(url + "/api/v1/gpu/fleet", timeout=30).json(), t0)
    req = dict(p["request"], training_script=script, dry_run=False, num_gpus=1, num_nodes=1,
               script_args=[*p["args"], "--metrics-url", url, *(extra_args or [])])
    r = httpx.post(url + "/api/v1/training/launch", json=req, timeout=60)
    r.raise_for_status()
    launch = r.json()
    job_id = launch["job_id"]
    during: List[Dict[str, Any]] = []
    job: Dict[str, Any] = {}
    while time.time() - t0 < p["timeout_s"]:
        job = httpx.get(f"{url}/api/v1/training/jobs/{job_id}", timeout=10).json()
        if job.get("status") in ("succeeded", "failed", "cancelled", "nan_halt", "preempted"):
            break
        try:
            during.append(_fleet_dev(httpx.get(url + "/api/v1/gpu/fleet", timeout=30).json(), t0))
        except httpx.HTTPError:
            pass
        time.sleep(poll_s)
    summary = {}
    for _ in range(40):  # metrics are pushed asynchronously by the trainer
        s = httpx.get(f"{url}/api/v1/monitoring/summary/{job_id}", timeout=10)
        if s.status_code == 200:
            summary = s.json()
            if summary.get("total_steps", 0) >= int(p["args"][p["args"].index("--steps") + 1]):
                break
        time.sleep(0.25)
    curve = httpx.get(f"{url}/api/v1/monitoring/loss-curve/{job_id}", timeout=10)
    after = _fleet_dev(httpx.get(url + "/api/v1/gpu/fleet", timeout=30).json(), t0)
    peak = max(during, key=lambda d: d.get("memory_used_mib") or 0) if during else None
    log_tail = ""
    if job.get("log_path") and os.path.exists(job["log_path"]):
        with open(job["log_path"]) as f:
            log_tail = f.read()[-6000:]
    return {"preset": preset, "request": {k: v for k, v in req.items() if k != "training_script"},
            "launch": launch, "job": {k: job.get(k) for k in ("job_id", "status", "exit_codes", "restarts", "events",
                                                               "pid", "log_path")},
            "elapsed_s": round(time.time() - t0, 1), "monitoring_summary": summary,
            "loss_curve": curve.json() if curve.status_code == 200 else None,
            "fleet": {"before": before, "peak_during": peak, "after": after, "samples": len(during)},
            "log_tail": log_tail}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--preset", default="llama-tiny", choices=sorted(PRESETS))
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    os.environ.setdefault("DLGM_TELEMETRY_INTERVAL_S", "0")
    with Server() as srv:
        rec = run(a.preset, srv.url)
    rec["recorded_at"] = time.strftime("%Y-%m-%dT%H:%M:%S")
    text = json.dumps(rec, indent=1, default=str)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            f.write(text)
    print(json.dumps({k: rec[k] for k in ("preset", "elapsed_s")} | {"status": rec["job"]["status"],
                     "steps": rec["monitoring_summary"].get("total_steps"),
                     "peak_hbm_mib": (rec["fleet"]["peak_during"] or {}).get("memory_used_mib")}))
    return 0 if rec["job"]["status"] == "succeeded" else 1


if __name__ == "__main__":
    sys.exit(main())
