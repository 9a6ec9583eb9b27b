"""DeepSpeed-schema JSON -> EngineConfig (engine/dsconfig.py): every key the reference's generator emits
(``ai_engine/deepspeed_launcher.py:124-238``) lands on the engine knob that implements it."""
import torch

from distributed_llm_training_gpu_manager_amd.engine.dsconfig import engine_config_from_ds
from distributed_llm_training_gpu_manager_amd.launcher.config import generate_config, presets


def test_presets_map_onto_engine():
    for name, pc in presets().items():
        ds = generate_config(pc)
        cfg, notes = engine_config_from_ds(ds, seq_len=4096)
        zo = ds["zero_optimization"]
        assert cfg.zero_stage == zo["stage"], name
        assert cfg.micro_batch_size == ds["train_micro_batch_size_per_gpu"]
        assert cfg.grad_accum == ds["gradient_accumulation_steps"]
        assert cfg.grad_clip == ds["gradient_clipping"]
        if zo["stage"] < 3:
            continue
        assert cfg.max_live_parameters == zo["stage3_max_live_parameters"]
        assert cfg.max_reuse_distance == zo["stage3_max_reuse_distance"]
        assert cfg.prefetch_bucket_size == zo["stage3_prefetch_bucket_size"]
        off = zo.get("offload_optimizer", {})
        assert cfg.offload_optimizer == off.get("device", "none")
        if "buffer_count" in off:
            assert cfg.offload_buffer_count == off["buffer_count"]
        assert cfg.offload_param == zo.get("offload_param", {}).get("device", "none")
        assert cfg.param_persistence_threshold == zo["stage3_param_persistence_threshold"]
        assert cfg.prescale_gradients == ds["prescale_gradients"]
        assert cfg.gradient_predivide_factor == ds["gradient_predivide_factor"]
        assert not any("not needed" in n or "not applicable" in n for n in notes)


def test_aio_and_mi355x_blocks():
    ds = {"zero_optimization": {"stage": 2, "offload_optimizer": {"device": "nvme", "nvme_path": "/nvme",
                                                                  "buffer_count": 6}},
          "aio": {"block_size": 1 << 20, "queue_depth": 4, "thread_count": 2},
          "communication_data_type": "fp16",
          "mi355x": {"expert_parallel_size": 2, "sequence_parallel_size": 4, "comm_dtype": "fp32"}}
    cfg, notes = engine_config_from_ds(ds, seq_len=1024)
    assert (cfg.offload_optimizer, cfg.nvme_path, cfg.offload_buffer_count) == ("nvme", "/nvme", 6)
    assert (cfg.aio_threads, cfg.aio_block_size) == (8, 1 << 20)
    assert (cfg.expert_parallel_size, cfg.sequence_parallel_size) == (2, 4)
    assert engine_config_from_ds({"mi355x": {"local_grad_accum": False}}, 64)[0].local_grad_accum is False
    assert engine_config_from_ds({"mi355x": {"hip_graphs": True}}, 64)[0].hip_graphs is True
    assert cfg.hip_graphs is False
    assert cfg.comm_dtype == torch.float32
    assert any("A20" in n for n in notes)


def test_gather_16bit_weights_key_controls_module_capture(tmp_path):
    """zero_optimization.stage3_gather_16bit_weights_on_model_save (DeepSpeed default False) decides whether a
    stage-3 save gathers the 16-bit module into mp_rank_00_model_states.pt."""
    from distributed_llm_training_gpu_manager_amd.ckpt.checkpoint import AsyncCheckpointer
    from distributed_llm_training_gpu_manager_amd.models import get_config
    from distributed_llm_training_gpu_manager_amd.parallel.zero import ZeroEngine
    base = {"zero_optimization": {"stage": 3}, "train_micro_batch_size_per_gpu": 1}
    cfg, _ = engine_config_from_ds(base, seq_len=32)
    assert cfg.gather_16bit_weights_on_model_save is False
    for flag in (False, True):
        ds = {**base, "zero_optimization": {"stage": 3, "stage3_gather_16bit_weights_on_model_save": flag}}
        cfg, _ = engine_config_from_ds(ds, seq_len=32)
        assert cfg.gather_16bit_weights_on_model_save is flag
        cfg.init_device = "cpu"
        eng = ZeroEngine(get_config("llama-tiny"), cfg, torch.device("cpu"))
        d = tmp_path / str(flag)
        ck = AsyncCheckpointer(eng, str(d), shm=False)
        ck.save(1, {"step": 1}, blocking=True)
        ck.close()
        meta = torch.load(d / "global_step1" / "mp_rank_00_model_states.pt", weights_only=True)
        assert (meta.get("module") is not None) is flag


def test_offload_param_nvme_path_is_its_own():
    ds = {"zero_optimization": {"stage": 3, "offload_optimizer": {"device": "nvme", "nvme_path": "/nvme0"},
                                "offload_param": {"device": "nvme", "nvme_path": "/nvme1"}}}
    cfg, _ = engine_config_from_ds(ds, seq_len=32)
    assert cfg.nvme_path == "/nvme0" and cfg.param_nvme_path == "/nvme1"
