"""Code written against the reference's ``ai_engine`` package imports unchanged."""
import importlib


def test_reference_import_surface():
    ae = importlib.import_module("ai_engine")
    for name in ["GPUManager", "GPUDevice", "GPUFleetStatus", "DeepSpeedLauncher", "DeepSpeedConfig",
                 "LossSpikeMonitor", "TrainingMetrics", "SpikeAlert"]:
        assert hasattr(ae, name), name
    dl = importlib.import_module("ai_engine.deepspeed_launcher")
    for name in ["ZeROStage", "OffloadDevice", "DeepSpeedConfig", "LaunchResult", "DeepSpeedLauncher"]:
        assert hasattr(dl, name), name
    gm = importlib.import_module("ai_engine.gpu_manager")
    for name in ["GPUHealthStatus", "GPUProcess", "GPUDevice", "GPUFleetStatus", "GPUManager"]:
        assert hasattr(gm, name), name
    lm = importlib.import_module("ai_engine.loss_monitor")
    for name in ["AlertSeverity", "SpikeAlert", "TrainingMetrics", "MonitorConfig", "MonitorState",
                 "LossSpikeMonitor"]:
        assert hasattr(lm, name), name
    assert hasattr(importlib.import_module("ai_engine.spot_resiliency"), "SpotInstanceResiliencyManager")


def test_reference_style_usage():
    from ai_engine import DeepSpeedConfig, DeepSpeedLauncher, LossSpikeMonitor, TrainingMetrics

    launcher = DeepSpeedLauncher()
    cfg = DeepSpeedConfig(model_name="m", training_script="train.py")
    ds = launcher.generate_config(cfg)
    assert ds["zero_optimization"]["stage"] == 3
    mon = LossSpikeMonitor()
    assert mon.ingest(TrainingMetrics(step=1, loss=2.0)) == []
    alerts = mon.ingest(TrainingMetrics(step=2, loss=float("nan")))
    assert alerts and alerts[0].alert_type == "divergence"
