"""Per-job loss-monitor endpoints (reference ``backend/routers/monitoring.py``).

Fixes: thread-safe registry; NaN / Inf values are serialised as strings instead of
crashing the JSON encoder (A14: NaN loss and a fresh monitor's ``best_loss=inf``
gave HTTP 500); re-creating an existing monitor reports the config actually in
use (A15).
"""
import threading
from typing import Dict, List, Optional

from fastapi import APIRouter, HTTPException
from fastapi.responses import JSONResponse
from pydantic import BaseModel

from distributed_llm_training_gpu_manager_amd.health.loss_monitor import (
    LossSpikeMonitor, MonitorConfig, TrainingMetrics, json_safe)

from distributed_llm_training_gpu_manager_amd.utils import metrics as prom

router = APIRouter()
_monitors: Dict[str, LossSpikeMonitor] = {}
_lock = threading.Lock()


def _safe(payload) -> JSONResponse:
    return JSONResponse(content=json_safe(payload))


def _get_or_create_monitor(job_id: str, config: Optional[MonitorConfig] = None) -> LossSpikeMonitor:
    with _lock:
        if job_id not in _monitors:
            _monitors[job_id] = LossSpikeMonitor(config)
        return _monitors[job_id]


class MonitorCreateRequest(BaseModel):
    job_id: str
    window_size: int = 100
    spike_sigma_threshold: float = 3.0
    divergence_threshold: float = 1e6
    plateau_patience: int = 500
    gradient_norm_threshold: float = 100.0


class MetricsIngestRequest(BaseModel):
    job_id: str
    metrics: List[TrainingMetrics]


class SingleMetricRequest(BaseModel):
    job_id: str
    step: int
    loss: float
    learning_rate: float = 0.0
    gradient_norm: float = 0.0
    throughput_samples_per_sec: float = 0.0
    gpu_memory_used_mib: int = 0


@router.post("/create")
def create_monitor(request: MonitorCreateRequest):
    config = MonitorConfig(window_size=request.window_size, spike_sigma_threshold=request.spike_sigma_threshold,
                           divergence_threshold=request.divergence_threshold,
                           plateau_patience=request.plateau_patience,
                           gradient_norm_threshold=request.gradient_norm_threshold)
    with _lock:
        existed = request.job_id in _monitors
    monitor = _get_or_create_monitor(request.job_id, config)
    return _safe({"job_id": request.job_id, "status": "exists" if existed else "created",
                  "config": monitor.config.model_dump()})


@router.post("/ingest")
def ingest_metrics(request: MetricsIngestRequest):
    monitor = _get_or_create_monitor(request.job_id)
    alerts = []
    for m in request.metrics:
        alerts.extend(monitor.ingest(m))
        _observe(request.job_id, m)
    for a in alerts:
        prom.observe_alert(request.job_id, str(getattr(a, "alert_type", "unknown")))
    return _safe({"job_id": request.job_id, "ingested": len(request.metrics), "alerts_triggered": len(alerts),
                  "alerts": [a.model_dump() for a in alerts]})


@router.post("/ingest/single")
def ingest_single_metric(request: SingleMetricRequest):
    monitor = _get_or_create_monitor(request.job_id)
    m = TrainingMetrics(
        step=request.step, loss=request.loss, learning_rate=request.learning_rate,
        gradient_norm=request.gradient_norm, throughput_samples_per_sec=request.throughput_samples_per_sec,
        gpu_memory_used_mib=request.gpu_memory_used_mib)
    alerts = monitor.ingest(m)
    _observe(request.job_id, m)
    for a in alerts:
        prom.observe_alert(request.job_id, str(getattr(a, "alert_type", "unknown")))
    return _safe({"job_id": request.job_id, "step": request.step, "alerts": [a.model_dump() for a in alerts],
                  "healthy": len(alerts) == 0})


def _observe(job_id: str, m: TrainingMetrics) -> None:
    prom.observe_training(job_id, {"loss": m.loss, "grad_norm": m.gradient_norm, "learning_rate": m.learning_rate,
                                   "throughput": m.throughput_samples_per_sec, "step": m.step,
                                   "gpu_memory_used": (m.gpu_memory_used_mib or 0) / 1024.0})


def _require(job_id: str) -> LossSpikeMonitor:
    with _lock:
        m = _monitors.get(job_id)
    if m is None:
        raise HTTPException(status_code=404, detail=f"No monitor for job '{job_id}'")
    return m


@router.get("/summary/{job_id}")
def get_monitor_summary(job_id: str):
    return _safe(_require(job_id).get_summary())


@router.get("/loss-curve/{job_id}")
def get_loss_curve(job_id: str):
    return _safe(_require(job_id).get_loss_curve())


@router.delete("/reset/{job_id}")
def reset_monitor(job_id: str):
    _require(job_id).reset()
    return {"job_id": job_id, "status": "reset"}


@router.get("/jobs")
def list_monitored_jobs():
    with _lock:
        items = list(_monitors.items())
    return _safe({"active_jobs": len(items),
                  "jobs": [{"job_id": j, "total_steps": m.state.total_steps, "total_alerts": m.state.alert_count,
                            "best_loss": m.state.best_loss} for j, m in items]})
