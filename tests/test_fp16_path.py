"""fp16 compute path (DeepSpeed "fp16" block, reference deepspeed_launcher.py:48-51, 173-183): the engine
computes in fp16 (gathered parameters, activations, gradients), keeps fp32 master weights, and the dynamic
loss scaler skips the step and backs off when the scaled fp16 gradients overflow."""
import pytest
import torch

from distributed_llm_training_gpu_manager_amd.models import get_config
from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine


def _engine(device, **kw):
    mc = get_config("llama-tiny")
    ec = EngineConfig(zero_stage=3, micro_batch_size=2, seq_len=64, grad_accum=1, lr=3e-3, scheduler="constant",
                      init_device="cpu", grad_clip=1.0, fp16=True, **kw)
    return ZeroEngine(mc, ec, torch.device(device)), mc


def _batch(mc, device, seed):
    g = torch.Generator().manual_seed(seed)
    t = torch.randint(0, mc.vocab_size, (2, 65), generator=g)
    return [(t[:, :-1].to(device), t[:, 1:].to(device))]


def _run(device):
    eng, mc = _engine(device, initial_scale_power=24, loss_scale_window=1000, hysteresis=1)
    assert eng.dtype == torch.float16 and eng.p16_shard.dtype == torch.float16
    scales, losses = [], []
    master0 = eng.master.clone()
    for i in range(12):
        m = eng.train_step(_batch(mc, device, 0))
        scales.append(eng.scaler.scale)
        losses.append(float(m["loss"]))
    # 2^24 overflows the fp16 gradients: the first steps are skipped and the scale halves each time
    assert scales[0] < 2.0 ** 24 and scales[1] < scales[0], scales
    assert torch.isfinite(eng.master).all()
    assert not torch.equal(eng.master, master0)  # once the scale is in range the steps apply
    assert losses[-1] < losses[0] - 0.05, losses
    return eng


def test_fp16_engine_loss_scaler_backs_off_cpu():
    _run("cpu")


@pytest.mark.gpu
def test_fp16_engine_loss_scaler_backs_off_gpu():
    eng = _run("cuda")
    # the compute copy that the kernels consumed is fp16, refreshed from the fp32 master by the optimizer
    assert torch.allclose(eng.p16_shard.float(), eng.master.half().float())
