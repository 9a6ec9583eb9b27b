"""LossSpikeMonitor: reference behaviour (goldens from the reference code) + the documented fixes."""
import json
import math
import os

import pytest

from distributed_llm_training_gpu_manager_amd.health.loss_monitor import (
    LossSpikeMonitor, MonitorConfig, TrainingMetrics, json_safe)

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "fixtures", "reference_golden", "loss_monitor.json")))


@pytest.mark.parametrize("case", sorted(GOLD))
def test_matches_reference_sequence(case):
    rec = GOLD[case]
    mon = LossSpikeMonitor(MonitorConfig(**rec["config"]))
    alerts = []
    for m in rec["metrics"]:
        for a in mon.ingest(TrainingMetrics(**m)):
            d = a.model_dump(mode="json")
            d.pop("timestamp")
            d["alert_id"] = d["alert_id"].rsplit("_", 1)[0]
            alerts.append(d)
    assert len(alerts) == len(rec["alerts"])
    for got, exp in zip(alerts, rec["alerts"]):
        for k in ("alert_id", "severity", "alert_type", "step", "message", "remediation"):
            assert got[k] == exp[k], (k, got[k], exp[k])
        for k in ("metric_value", "threshold", "rolling_mean", "rolling_std"):
            assert math.isclose(got[k], exp[k], rel_tol=1e-9, abs_tol=1e-9), (k, got[k], exp[k])
    summ = mon.get_summary()
    for k, v in rec["summary"].items():
        if isinstance(v, float):
            assert math.isclose(summ[k], v, rel_tol=1e-9), k
        else:
            assert summ[k] == v, k
    assert mon.get_loss_curve() == rec["curve"]


def test_nan_alert_is_stored_and_counted():
    mon = LossSpikeMonitor()
    for i in range(5):
        mon.ingest(TrainingMetrics(step=i, loss=1.0))
    a = mon.ingest(TrainingMetrics(step=5, loss=float("nan")))
    assert a[0].alert_type == "divergence" and a[0].severity == "critical"
    assert mon.state.alert_count == 1 and mon.get_summary()["alert_counts_by_type"] == {"divergence": 1}
    assert mon.get_summary()["current_loss"] == 1.0  # NaN never entered the window


def test_max_alerts_per_type_cap():
    mon = LossSpikeMonitor(MonitorConfig(max_alerts_per_type=3, divergence_threshold=10))
    for i in range(10):
        mon.ingest(TrainingMetrics(step=i, loss=100.0))  # divergence has no cooldown
    assert len([a for a in mon._all_alerts if a.alert_type == "divergence"]) == 3
    assert mon.state.alert_count == 10


def test_device_stats_feed_and_reset():
    mon = LossSpikeMonitor()
    a = mon.ingest_device_stats(7, grad_sumsq=1.0, nonfinite=3)
    assert a and "NaN/Inf trap" in a[0].message
    assert mon.ingest_device_stats(8, grad_sumsq=4.0, nonfinite=0, loss=2.0) == []
    mon.reset()
    assert mon.state.total_steps == 0 and mon.get_loss_curve()["steps"] == []


def test_json_safe():
    assert json_safe({"a": float("nan"), "b": [float("inf"), -float("inf"), 1.5]}) == \
        {"a": "NaN", "b": ["Infinity", "-Infinity", 1.5]}
