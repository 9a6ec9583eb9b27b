"""DeepSpeed-schema config generation parity with the reference (goldens recorded from its own code)."""
import json
import os
import shlex

import pytest

from distributed_llm_training_gpu_manager_amd.launcher.config import (
    DeepSpeedConfig, OffloadDevice, ZeROStage, generate_config, presets)
from distributed_llm_training_gpu_manager_amd.launcher.launcher import DeepSpeedLauncher, ZeroLauncher

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "fixtures", "reference_golden", "generate_config.json")))


def _expected(ref: dict, cfg: DeepSpeedConfig) -> dict:
    """Reference JSON with the documented deviations applied (A20 comm dtype, A21 elasticity, A22 nvme_path)."""
    exp = json.loads(json.dumps(ref))
    if cfg.bf16_enabled and exp.get("communication_data_type") == "fp16":
        exp["communication_data_type"] = "bf16"
    if "elasticity" in exp:
        exp["elasticity"]["micro_batch_sizes"] = [cfg.train_micro_batch_size_per_gpu]
        exp["elasticity"]["version"] = 0.2
    zo = exp["zero_optimization"]
    for key in ("offload_optimizer", "offload_param"):
        if key in zo and zo[key]["device"] == "nvme":
            zo[key]["nvme_path"] = "/local_nvme"
    return exp


@pytest.mark.parametrize("case", sorted(GOLD))
def test_generate_config_matches_reference(case):
    rec = GOLD[case]
    cfg = DeepSpeedConfig(**rec["config"])
    assert generate_config(cfg) == _expected(rec["ds_config"], cfg)


def test_reference_presets_unchanged():
    p = presets()
    for name in ("7b", "13b", "70b"):
        assert p[name].model_dump(mode="json", exclude={"nvme_path", "mi355x"}) == GOLD[f"preset_{name}"]["config"]
        assert p[name].effective_batch_size == {"7b": 128, "13b": 256, "70b": 1024}[name]


def test_mi355x_presets_fit_hbm_without_offload():
    p = presets()
    for name in ("llama3-8b", "llama3-70b", "mixtral-8x7b"):
        assert p[name].offload_optimizer == OffloadDevice.NONE and p[name].offload_param == OffloadDevice.NONE
        assert generate_config(p[name])["mi355x"]["nan_trap"] is True


def test_launch_dry_run_contract(tmp_path):
    L = ZeroLauncher()
    cfg = DeepSpeedConfig(model_name="m", num_gpus=4, num_nodes=2, train_micro_batch_size_per_gpu=2,
                          gradient_accumulation_steps=3, bf16_enabled=True, fp16_enabled=False)
    r = L.launch(cfg, "my train.py", ["--foo", "a b"], dry_run=True)
    assert r.status == "dry_run" and r.num_gpus == 8 and r.num_nodes == 2 and r.effective_batch_size == 48
    assert r.job_id.startswith("ds_m_")
    assert r.details == {"zero_stage": 3, "offload_optimizer": "cpu", "offload_param": "cpu", "precision": "bf16",
                         "activation_checkpointing": True, "dry_run": True}
    argv = shlex.split(r.command)
    assert "my train.py" in argv and "a b" in argv  # A17: spaces survive
    assert "--nproc-per-node=4" in argv and "--nnodes=2" in argv
    assert any(a.startswith("--deepspeed_config=") for a in argv)
    assert json.load(open(r.config_path))["bf16"] == {"enabled": True}
    # A19: two launches in the same second get different ids
    assert L.launch(cfg, "t.py", dry_run=True).job_id != L.launch(cfg, "t.py", dry_run=True).job_id


def test_launch_missing_binary_reports_failed():
    L = DeepSpeedLauncher(deepspeed_path="/nonexistent/launcher")
    r = L.launch(DeepSpeedConfig(), "train.py", dry_run=False)
    assert r.status == "failed" and "error" in r.details


def test_write_config_and_command(tmp_path):
    L = ZeroLauncher()
    cfg = DeepSpeedConfig(zero_stage=ZeROStage.OPTIMIZER_STATE)
    path = L.write_config(cfg, str(tmp_path / "c.json"))
    assert json.load(open(path))["zero_optimization"]["stage"] == 1
    cmd = L.build_launch_command(cfg, "train.py", None, path)
    assert cmd.endswith(f"train.py --deepspeed_config={path}")
