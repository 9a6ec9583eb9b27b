"""Ulysses sequence parallelism (parallel/sp.py) on gloo, world 2.

Two ranks each holding half of every sequence must produce the loss and the gradients of one
process training on the whole sequences: RoPE at global positions, causal attention over the
full sequence through the head/sequence all-to-all, exact adjoint in the backward.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_llm_training_gpu_manager_amd.models import get_config
from distributed_llm_training_gpu_manager_amd.parallel.comm import Comm
from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine

S_FULL = 64


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _tokens(mc):
    g = torch.Generator().manual_seed(31)
    return torch.randint(0, mc.vocab_size, (2, S_FULL + 1), generator=g)


def _cfg(stage, seq, sp):
    return EngineConfig(zero_stage=stage, micro_batch_size=2, seq_len=seq, grad_accum=1, lr=1e-2, scheduler="constant",
                        init_device="cpu", grad_clip=0.0, comm_dtype=torch.float32, sequence_parallel_size=sp)


def _worker(rank, world, port, stage, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mc = get_config("llama-tiny")
    S = S_FULL // world
    eng = ZeroEngine(mc, _cfg(stage, S, world), torch.device("cpu"), Comm())
    t = _tokens(mc)
    ids, lab = t[:, :-1], t[:, 1:]
    sl = slice(rank * S, (rank + 1) * S)
    loss = eng.micro_step(ids[:, sl].contiguous(), lab[:, sl].contiguous(), first=True, last=True)
    tot = torch.tensor([float(loss)])
    dist.all_reduce(tot)
    grads = eng.full_grads()
    if rank == 0:
        torch.save({"loss": float(tot) / (2 * S_FULL), "grads": grads}, out_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("stage", [0, 3])
def test_ulysses_world2_matches_full_sequence(tmp_path, stage):
    out = str(tmp_path / "sp.pt")
    mp.spawn(_worker, args=(2, _free_port(), stage, out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    mc = get_config("llama-tiny")
    eng = ZeroEngine(mc, _cfg(stage, S_FULL, 1), torch.device("cpu"))
    t = _tokens(mc)
    loss = float(eng.micro_step(t[:, :-1].contiguous(), t[:, 1:].contiguous(), first=True, last=True)) / (2 * S_FULL)
    assert abs(loss - got["loss"]) < 1e-3 * max(1.0, abs(loss)), (loss, got["loss"])
    ref = eng.full_grads()
    assert set(ref) == set(got["grads"])
    for k, v in ref.items():
        err = float((got["grads"][k] - v).abs().max() / v.abs().max().clamp_min(1e-8))
        assert err < 2e-2, (k, err)


def _train_worker(rank, world, port, out_path):
    """The training script end to end with --sequence-parallel 2 (gloo): runs and learns."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from distributed_llm_training_gpu_manager_amd.engine.trainer import Trainer, parse_args

    args = parse_args(["--model", "llama-tiny", "--seq-len", "64", "--steps", "4", "--device", "cpu",
                       "--sequence-parallel", "2", "--zero-stage", "3", "--lr", "3e-3", "--log-json", out_path])
    t = Trainer(args)
    assert t.ecfg.seq_len == 32 and t.engine.sp_size == 2
    assert t.run() == 0


def test_trainer_sequence_parallel_world2(tmp_path):
    import json

    out = str(tmp_path / "log.json")
    mp.spawn(_train_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    log = json.load(open(out))["log"]
    assert len(log) == 4 and all(r["loss"] == r["loss"] for r in log)
