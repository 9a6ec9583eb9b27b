"""Prometheus exposition for training + fleet metrics (the reference keeps
metrics in per-process dicts only). Served by the control plane at ``GET /metrics``."""
from __future__ import annotations

from typing import Any, Dict, Optional

from prometheus_client import CollectorRegistry, Gauge, generate_latest
from prometheus_client import CONTENT_TYPE_LATEST  # noqa: F401  (re-exported for the router)

REGISTRY = CollectorRegistry()
_TRAIN = {
    "loss": Gauge("dlgm_train_loss", "latest training loss", ["job"], registry=REGISTRY),
    "grad_norm": Gauge("dlgm_train_grad_norm", "latest global gradient norm", ["job"], registry=REGISTRY),
    "learning_rate": Gauge("dlgm_train_lr", "latest learning rate", ["job"], registry=REGISTRY),
    "throughput": Gauge("dlgm_train_tokens_per_second", "tokens/s (whole job)", ["job"], registry=REGISTRY),
    "step": Gauge("dlgm_train_step", "latest optimizer step", ["job"], registry=REGISTRY),
    "gpu_memory_used": Gauge("dlgm_train_gpu_memory_gib", "peak HBM in use (GiB)", ["job"], registry=REGISTRY),
}
_ALERTS = Gauge("dlgm_train_alerts_total", "loss-monitor alerts raised", ["job", "type"], registry=REGISTRY)
_GPU = {
    "temperature": Gauge("dlgm_gpu_temperature_celsius", "junction (hotspot) temperature", ["gpu"], registry=REGISTRY),
    "hbm_temperature": Gauge("dlgm_gpu_hbm_temperature_celsius", "max HBM stack temperature", ["gpu"],
                             registry=REGISTRY),
    "utilization": Gauge("dlgm_gpu_utilization_percent", "GFX activity", ["gpu"], registry=REGISTRY),
    "memory_used": Gauge("dlgm_gpu_memory_used_mib", "VRAM used", ["gpu"], registry=REGISTRY),
    "power": Gauge("dlgm_gpu_power_watts", "socket power", ["gpu"], registry=REGISTRY),
}


def observe_training(job_id: str, m: Dict[str, Any]) -> None:
    for k, g in _TRAIN.items():
        v = m.get(k)
        if isinstance(v, (int, float)) and v == v:  # skip None / NaN
            g.labels(job=job_id).set(float(v))


def observe_alert(job_id: str, alert_type: str) -> None:
    _ALERTS.labels(job=job_id, type=alert_type).inc()


def observe_fleet(fleet: Optional[Any]) -> None:
    if fleet is None:
        return
    for d in getattr(fleet, "gpus", []) or []:
        lab = str(getattr(d, "index", "?"))
        for attr, g in (("temperature_celsius", _GPU["temperature"]), ("gpu_utilization_pct", _GPU["utilization"]),
                        ("memory_used_mib", _GPU["memory_used"]), ("power_draw_watts", _GPU["power"])):
            v = getattr(d, attr, None)
            if isinstance(v, (int, float)):
                g.labels(gpu=lab).set(float(v))
        hbm = getattr(d, "hbm_temperature_celsius", None)
        if isinstance(hbm, (int, float)):
            _GPU["hbm_temperature"].labels(gpu=lab).set(float(hbm))


def render() -> bytes:
    return generate_latest(REGISTRY)
