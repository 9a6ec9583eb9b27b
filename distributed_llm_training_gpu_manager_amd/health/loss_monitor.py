"""Training-health monitor: loss spikes, divergence (NaN/Inf/huge), plateaus, gradient
explosions and learning-rate anomalies.

Behaviour and wire format follow the reference ``ai_engine/loss_monitor.py``
(rule order ``:111-243``, defaults ``:58-66``, message formats, ``alert_id`` scheme
``:287``, cooldown ``:301-304``, summary / loss-curve payloads ``:245-271``), so a
client of the reference API sees the same alerts. The statistics are kept as
running sums over the window (O(1) per step instead of ``statistics.stdev`` over
the deque at every step).

Documented fixes:
  * A8  -- a NaN/Inf loss alert is stored and counted (the reference returns before
    both), and the non-finite value never enters the rolling window;
  * A11 -- ``max_alerts_per_type`` is enforced on the stored history (oldest dropped);
  * A14 -- :func:`json_safe` maps NaN/Inf floats to strings for the REST layer.

On-device integration: :meth:`LossSpikeMonitor.ingest_device_stats` consumes the
engine's ``grad_stats`` buffer (sum g^2, non-finite count) asynchronously, so a NaN
gradient raises a ``divergence`` alert without the training loop ever syncing.
"""
from __future__ import annotations

import math
from collections import deque
from enum import Enum
from typing import Any, Deque, Dict, List, Optional

from pydantic import BaseModel, Field

from ..launcher.config import utcnow


class AlertSeverity(str, Enum):
    INFO = "info"
    WARNING = "warning"
    CRITICAL = "critical"


class SpikeAlert(BaseModel):
    """Alert triggered by the loss monitor."""
    alert_id: str
    severity: AlertSeverity
    alert_type: str = Field(..., description="spike | divergence | plateau | gradient_explosion | lr_anomaly")
    step: int
    message: str
    metric_value: float
    threshold: float
    rolling_mean: float
    rolling_std: float
    remediation: List[str] = Field(default_factory=list)
    timestamp: str = Field(default_factory=lambda: utcnow().isoformat())


class TrainingMetrics(BaseModel):
    """Snapshot of training metrics at a single step."""
    step: int
    loss: float
    learning_rate: float = 0.0
    gradient_norm: float = 0.0
    throughput_samples_per_sec: float = 0.0
    gpu_memory_used_mib: int = 0
    epoch: Optional[int] = None
    timestamp: str = Field(default_factory=lambda: utcnow().isoformat())
    # additions (optional, ignored by reference clients)
    tokens_per_sec: Optional[float] = None
    mfu: Optional[float] = None


class MonitorConfig(BaseModel):
    """Configuration for the loss spike monitor (reference defaults)."""
    window_size: int = Field(default=100, description="Rolling window for statistics")
    spike_sigma_threshold: float = Field(default=3.0, description="Std devs for spike detection")
    divergence_threshold: float = Field(default=1e6, description="Loss considered diverged")
    plateau_patience: int = Field(default=500, description="Steps without improvement for plateau")
    plateau_min_delta: float = Field(default=1e-4, description="Minimum improvement to reset plateau")
    gradient_norm_threshold: float = Field(default=100.0, description="Max gradient norm before alert")
    lr_spike_ratio: float = Field(default=10.0, description="LR jump ratio for alert")
    max_alerts_per_type: int = Field(default=50, description="Max alerts to store per type")
    cooldown_steps: int = Field(default=20, description="Min steps between same-type alerts")


class MonitorState(BaseModel):
    """Serializable monitor state for persistence."""
    total_steps: int = 0
    best_loss: float = float("inf")
    best_loss_step: int = 0
    plateau_counter: int = 0
    alert_count: int = 0
    last_alert_step: Dict[str, int] = Field(default_factory=dict)


class _Window:
    """Fixed-size window with running sum / sum of squares (sample std, like ``statistics.stdev``)."""

    def __init__(self, n: int):
        self.q: Deque[float] = deque(maxlen=max(1, n))
        self.s = 0.0
        self.ss = 0.0

    def append(self, x: float) -> None:
        if len(self.q) == self.q.maxlen:
            old = self.q[0]
            self.s -= old
            self.ss -= old * old
        self.q.append(x)
        self.s += x
        self.ss += x * x

    def __len__(self) -> int:
        return len(self.q)

    def mean(self) -> float:
        return self.s / len(self.q)

    def stdev(self) -> float:
        n = len(self.q)
        if n < 2:
            return 0.0
        m = self.s / n
        var = max(0.0, (self.ss - n * m * m) / (n - 1))
        # exact recomputation when cancellation makes the running form unreliable
        if var < 1e-12 * max(1.0, m * m):
            var = sum((x - m) ** 2 for x in self.q) / (n - 1)
        return math.sqrt(var)

    def clear(self) -> None:
        self.q.clear()
        self.s = self.ss = 0.0

    def values(self) -> List[float]:
        return list(self.q)


class LossSpikeMonitor:
    """Real-time training loss monitor with anomaly detection (reference API)."""

    def __init__(self, config: Optional[MonitorConfig] = None):
        self.config = config or MonitorConfig()
        self.state = MonitorState()
        self._loss_history = _Window(self.config.window_size)
        self._grad_history = _Window(self.config.window_size)
        self._lr_history = _Window(self.config.window_size)
        self._all_metrics: List[TrainingMetrics] = []
        self._all_alerts: List[SpikeAlert] = []
        self._type_counts: Dict[str, int] = {}

    # ------------------------------------------------------------------ ingest
    def ingest(self, metrics: TrainingMetrics) -> List[SpikeAlert]:
        alerts: List[SpikeAlert] = []
        cfg = self.config
        self.state.total_steps += 1
        self._all_metrics.append(metrics)
        loss = metrics.loss

        # 1. divergence: NaN / Inf
        if math.isnan(loss) or math.isinf(loss):
            alerts.append(self._create_alert(
                "divergence", AlertSeverity.CRITICAL, metrics.step, loss, 0, 0, 0,
                f"Loss diverged at step {metrics.step}: {loss}",
                ["Immediately reduce learning rate by 10x",
                 "Check for data corruption in current batch",
                 "Enable gradient clipping if not already active",
                 "Restore from last checkpoint and retry with lower LR"]))
            self._store(alerts)  # A8: stored and counted; the window is not polluted
            return alerts

        if loss > cfg.divergence_threshold:
            alerts.append(self._create_alert(
                "divergence", AlertSeverity.CRITICAL, metrics.step, loss, cfg.divergence_threshold, 0, 0,
                f"Loss {loss:.4e} exceeds divergence threshold {cfg.divergence_threshold:.4e}",
                ["Reduce learning rate by 5-10x",
                 "Increase gradient clipping value",
                 "Check for numerical instability in model architecture"]))

        # 2. spike
        if len(self._loss_history) >= 10:
            mean = self._loss_history.mean()
            std = self._loss_history.stdev()
            threshold = mean + cfg.spike_sigma_threshold * max(std, 1e-8)
            if loss > threshold and self._can_alert("spike", metrics.step):
                sev = AlertSeverity.CRITICAL if loss > mean + 5 * max(std, 1e-8) else AlertSeverity.WARNING
                alerts.append(self._create_alert(
                    "spike", sev, metrics.step, loss, threshold, mean, std,
                    f"Loss spike at step {metrics.step}: {loss:.6f} "
                    f"(mean={mean:.6f}, std={std:.6f}, threshold={threshold:.6f})",
                    ["Monitor next 10 steps for recovery",
                     "If persistent, reduce learning rate",
                     "Check system logs for GPU errors or data issues",
                     "Consider reverting to previous checkpoint"]))

        # 3. plateau
        if loss < self.state.best_loss - cfg.plateau_min_delta:
            self.state.best_loss = loss
            self.state.best_loss_step = metrics.step
            self.state.plateau_counter = 0
        else:
            self.state.plateau_counter += 1
        if self.state.plateau_counter >= cfg.plateau_patience and self._can_alert("plateau", metrics.step):
            alerts.append(self._create_alert(
                "plateau", AlertSeverity.WARNING, metrics.step, loss, self.state.best_loss,
                float(self.state.plateau_counter), 0,
                f"Training plateau: no improvement for {self.state.plateau_counter} steps "
                f"(best={self.state.best_loss:.6f} at step {self.state.best_loss_step})",
                ["Consider reducing learning rate (cosine annealing or step decay)",
                 "Try increasing model capacity or data augmentation",
                 "Evaluate if training has converged (check validation metrics)",
                 "Experiment with different optimizer (switch AdamW ↔ LAMB)"]))

        # 4. gradient explosion
        gn = metrics.gradient_norm
        if gn > 0 or math.isnan(gn) or math.isinf(gn):
            if (not math.isfinite(gn) or gn > cfg.gradient_norm_threshold) and \
                    self._can_alert("gradient_explosion", metrics.step):
                alerts.append(self._create_alert(
                    "gradient_explosion", AlertSeverity.WARNING, metrics.step, gn, cfg.gradient_norm_threshold,
                    self._grad_history.mean() if len(self._grad_history) else 0, 0,
                    f"Gradient norm explosion at step {metrics.step}: {gn:.4f} > {cfg.gradient_norm_threshold}",
                    ["Reduce gradient clipping value",
                     "Lower learning rate",
                     "Check for exploding activations in specific layers"]))
            if math.isfinite(gn):
                self._grad_history.append(gn)

        # 5. learning-rate anomaly
        lr = metrics.learning_rate
        if lr > 0 and len(self._lr_history) >= 5:
            avg_lr = self._lr_history.mean()
            if lr > avg_lr * cfg.lr_spike_ratio and self._can_alert("lr_anomaly", metrics.step):
                alerts.append(self._create_alert(
                    "lr_anomaly", AlertSeverity.WARNING, metrics.step, lr, avg_lr * cfg.lr_spike_ratio, avg_lr, 0,
                    f"Learning rate jump at step {metrics.step}: {lr:.2e} (avg={avg_lr:.2e})",
                    ["Verify LR scheduler configuration",
                     "Check for warmup restart if using cosine with restarts"]))
        if lr > 0:
            self._lr_history.append(lr)

        self._loss_history.append(loss)
        self._store(alerts)
        return alerts

    def ingest_device_stats(self, step: int, grad_sumsq: float, nonfinite: float, lr: float = 0.0,
                            loss: Optional[float] = None) -> List[SpikeAlert]:
        """Feed the engine's on-device gradient statistics (read asynchronously by the NaN trap)."""
        if nonfinite > 0:
            a = self._create_alert(
                "divergence", AlertSeverity.CRITICAL, step, float("nan"), 0, 0, 0,
                f"Non-finite gradients at step {step}: {int(nonfinite)} elements (NaN/Inf trap)",
                ["Optimizer step was skipped on device",
                 "Restore from last checkpoint and retry with lower LR",
                 "Check for data corruption in current batch"])
            self._store([a])
            return [a]
        return self.ingest(TrainingMetrics(step=step, loss=loss if loss is not None else 0.0,
                                           learning_rate=lr, gradient_norm=math.sqrt(max(grad_sumsq, 0.0))))

    # ------------------------------------------------------------------ views
    def get_summary(self) -> Dict[str, Any]:
        loss_list = self._loss_history.values()
        return {
            "total_steps": self.state.total_steps,
            "best_loss": self.state.best_loss,
            "best_loss_step": self.state.best_loss_step,
            "current_loss": loss_list[-1] if loss_list else None,
            "rolling_mean": self._loss_history.mean() if loss_list else None,
            "rolling_std": self._loss_history.stdev() if len(loss_list) > 1 else None,
            "plateau_counter": self.state.plateau_counter,
            "total_alerts": self.state.alert_count,
            "recent_alerts": [a.model_dump() for a in self._all_alerts[-10:]],
            "alert_counts_by_type": self._count_alerts_by_type(),
        }

    def get_loss_curve(self) -> Dict[str, Any]:
        return {
            "steps": [m.step for m in self._all_metrics],
            "losses": [m.loss for m in self._all_metrics],
            "learning_rates": [m.learning_rate for m in self._all_metrics],
            "gradient_norms": [m.gradient_norm for m in self._all_metrics],
            "spike_steps": [a.step for a in self._all_alerts if a.alert_type == "spike"],
        }

    def reset(self) -> None:
        """Reset the monitor (e.g. after loading a checkpoint)."""
        self._loss_history.clear()
        self._grad_history.clear()
        self._lr_history.clear()
        self._all_metrics.clear()
        self._all_alerts.clear()
        self._type_counts.clear()
        self.state = MonitorState()

    # ------------------------------------------------------------------ internals
    def _store(self, alerts: List[SpikeAlert]) -> None:
        cap = self.config.max_alerts_per_type
        for a in alerts:
            self._all_alerts.append(a)
            self._type_counts[a.alert_type] = self._type_counts.get(a.alert_type, 0) + 1
            # A11: keep at most `cap` stored alerts per type (oldest dropped)
            same = [i for i, x in enumerate(self._all_alerts) if x.alert_type == a.alert_type]
            if cap > 0 and len(same) > cap:
                del self._all_alerts[same[0]]
        self.state.alert_count += len(alerts)

    def _create_alert(self, alert_type: str, severity: AlertSeverity, step: int, value: float, threshold: float,
                      mean: float, std: float, message: str, remediation: List[str]) -> SpikeAlert:
        alert = SpikeAlert(
            alert_id=f"{alert_type}_{step}_{utcnow().strftime('%H%M%S')}",
            severity=severity, alert_type=alert_type, step=step, message=message, metric_value=value,
            threshold=threshold, rolling_mean=mean, rolling_std=std, remediation=remediation)
        self.state.last_alert_step[alert_type] = step
        return alert

    def _can_alert(self, alert_type: str, step: int) -> bool:
        last = self.state.last_alert_step.get(alert_type, -999)
        return step - last >= self.config.cooldown_steps

    def _count_alerts_by_type(self) -> Dict[str, int]:
        return dict(self._type_counts)


def json_safe(obj: Any) -> Any:
    """Recursively replace non-finite floats (NaN / +-Inf) with strings (A14: no HTTP 500)."""
    if isinstance(obj, float):
        if math.isnan(obj):
            return "NaN"
        if math.isinf(obj):
            return "Infinity" if obj > 0 else "-Infinity"
        return obj
    if isinstance(obj, dict):
        return {k: json_safe(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [json_safe(v) for v in obj]
    if isinstance(obj, BaseModel):
        return json_safe(obj.model_dump())
    if isinstance(obj, Enum):
        return obj.value
    return obj
