"""Multi-process ZeRO equivalence on CPU/gloo (the "multi-node without a cluster" fake).

W=2 ranks x GA=1 (each rank a different micro-batch) must produce the same
parameters as W=1 x GA=2 over the same two micro-batches, for every ZeRO stage.
"""
import json
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_llm_training_gpu_manager_amd.models import get_config
from distributed_llm_training_gpu_manager_amd.parallel.comm import Comm
from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _data(model, steps, n_micro):
    mc = get_config(model)
    g = torch.Generator().manual_seed(11)
    return [[torch.randint(0, mc.vocab_size, (2, 33), generator=g) for _ in range(n_micro)] for _ in range(steps)]


def _cfg(stage, ga, comm_dtype=torch.float32):
    return EngineConfig(zero_stage=stage, micro_batch_size=2, seq_len=32, grad_accum=ga, lr=1e-2,
                        scheduler="constant", init_device="cpu", grad_clip=1.0, comm_dtype=comm_dtype)


def _worker(rank, world, port, model, stage, steps, out_path, comm_dtype=torch.float32):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    eng = ZeroEngine(get_config(model), _cfg(stage, 1, comm_dtype), torch.device("cpu"), Comm())
    losses, grads0 = [], None
    for mbs in _data(model, steps, world):
        t = mbs[rank]
        m = eng.train_step([(t[:, :-1], t[:, 1:])])
        losses.append(float(m["loss"]))
        if grads0 is None:
            grads0 = eng.full_grads()
    params = eng.full_params()
    if rank == 0:
        torch.save({"params": params, "losses": losses, "grads0": grads0}, out_path)
    dist.barrier()
    dist.destroy_process_group()


def _single(model, stage, steps):
    eng = ZeroEngine(get_config(model), _cfg(stage, 2), torch.device("cpu"))
    losses, grads0 = [], None
    for mbs in _data(model, steps, 2):
        m = eng.train_step([(t[:, :-1], t[:, 1:]) for t in mbs])
        losses.append(float(m["loss"]))
        if grads0 is None:
            grads0 = eng.full_grads()
    return eng.full_params(), losses, grads0


def _compare(got, ref_params, ref_grads0, steps, lr=1e-2):
    """Step-1 gradients must match tightly. Parameters after `steps` Adam steps are compared
    robustly: W=2 reduces bf16 per-rank gradients while W=1 accumulates fp32 in the GEMM, and Adam
    turns a sign flip of a near-zero gradient element into a full +-lr step."""
    for k, v in ref_grads0.items():
        err = float((got["grads0"][k] - v).abs().max() / v.abs().max().clamp_min(1e-8))
        assert err < 2e-2, ("grad", k, err)
    for k, v in ref_params.items():
        d = (got["params"][k] - v).abs()
        assert float(d.max()) <= 2 * lr * steps + 1e-3, ("param max", k, float(d.max()))
        assert float((d > 0.1 * lr).float().mean()) < 0.05, ("param frac", k)


@pytest.mark.parametrize("stage", [0, 1, 2, 3])
@pytest.mark.parametrize("model", ["llama-tiny"])
def test_zero_stage_world2_matches_single(tmp_path, stage, model):
    out = str(tmp_path / "w2.pt")
    mp.spawn(_worker, args=(2, _free_port(), model, stage, 2, out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    ref_params, _, ref_grads0 = _single(model, stage, 2)
    # the world-2 loss is rank 0's own micro-batch; compare gradients and parameters, which see both
    _compare(got, ref_params, ref_grads0, 2)


def test_gpt2_zero1_world2(tmp_path):
    """BASELINE config 1 shape: GPT-2 family under ZeRO-1 on gloo (tied embeddings)."""
    out = str(tmp_path / "g.pt")
    mp.spawn(_worker, args=(2, _free_port(), "gpt2-tiny", 1, 2, out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    ref_params, _, ref_grads0 = _single("gpt2-tiny", 1, 2)
    _compare(got, ref_params, ref_grads0, 2)


def _grad_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = ZeroEngine(get_config("llama-tiny"), _cfg(3, 1, torch.bfloat16), torch.device("cpu"), Comm())
    t = _data("llama-tiny", 1, world)[0][rank]
    eng.micro_step(t[:, :-1], t[:, 1:], first=True, last=True)
    shards = [torch.empty_like(eng.grad_shard) for _ in range(world)]
    dist.all_gather(shards, eng.grad_shard)
    if rank == 0:
        torch.save({"shards": shards}, out_path)
    dist.barrier()
    dist.destroy_process_group()


def test_zero3_world2_bf16_comm_gradients(tmp_path):
    """The GPU default path: bf16 reduce-scatter of each flat gradient segment, fp32 accumulation.

    Compared on the gradients (Adam amplifies the sign of near-cancelling grads, so parameters
    after a step are not a meaningful bf16-vs-fp32 comparison).
    """
    out = str(tmp_path / "b.pt")
    mp.spawn(_grad_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    shards = torch.load(out, weights_only=True)["shards"]
    eng = ZeroEngine(get_config("llama-tiny"), _cfg(3, 2), torch.device("cpu"))
    for i, t in enumerate(_data("llama-tiny", 1, 2)[0]):
        eng.micro_step(t[:, :-1], t[:, 1:], first=i == 0, last=i == 1)
    for g in eng.groups:
        ref = eng.grad_shard.narrow(0, g.shard_off, g.shard_numel)
        half = g.shard_numel // 2
        got = torch.cat([shards[r].narrow(0, g.shard_off // 2, half) for r in range(2)])
        err = float((got - ref).abs().max() / ref.abs().max().clamp_min(1e-8))
        assert err < 2e-2, (g.name, err)


def _ep_worker(rank, world, port, stage, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = _cfg(stage, 1)
    cfg.expert_parallel_size = world
    eng = ZeroEngine(get_config("mixtral-tiny"), cfg, torch.device("cpu"), Comm())
    init = eng.full_params()
    t = _data("mixtral-tiny", 1, world)[0][rank]
    eng.micro_step(t[:, :-1], t[:, 1:], first=True, last=True)
    grads = eng.full_grads()
    if rank == 0:
        torch.save({"params": init, "grads": grads}, out_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("stage", [1, 3])
def test_mixtral_expert_parallel_world2_matches_single(tmp_path, stage):
    """BASELINE config 5 plumbing: EP=2 all-to-all dispatch/combine == single-process MoE gradients.

    Init is identical (experts seeded by global index), and the accumulated gradients of every
    parameter -- dense ones reduce-scattered over the world, expert ones computed on the EP rank
    that owns them from tokens of both ranks -- match the single-process 2-micro-batch run.
    """
    out = str(tmp_path / "ep.pt")
    mp.spawn(_ep_worker, args=(2, _free_port(), stage, out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    eng = ZeroEngine(get_config("mixtral-tiny"), _cfg(stage, 2), torch.device("cpu"))
    ref_init = eng.full_params()
    for k, v in ref_init.items():
        assert torch.equal(got["params"][k], v), k
    for i, t in enumerate(_data("mixtral-tiny", 1, 2)[0]):
        eng.micro_step(t[:, :-1], t[:, 1:], first=i == 0, last=i == 1)
    ref = eng.full_grads()
    assert set(got["grads"]) == set(ref)
    for k, v in ref.items():
        err = float((got["grads"][k] - v).abs().max() / v.abs().max().clamp_min(1e-8))
        assert err < 2e-2, (k, err)


def _comm_bench_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import importlib.util

    spec = importlib.util.spec_from_file_location(
        "comm_bench", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "comm_bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    rows = mod.main(["--min-mb", "0.0625", "--max-mb", "0.125", "--iters", "2", "--warmup", "1", "--dtype", "fp32"])
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(rows, f)
    dist.barrier()
    dist.destroy_process_group()


def test_comm_bench_gloo_world2(tmp_path):
    out = str(tmp_path / "cb.json")
    mp.spawn(_comm_bench_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    with open(out) as f:
        rows = json.load(f)
    assert {r["op"] for r in rows} == {"all_gather", "reduce_scatter", "all_reduce", "all_to_all"}
    assert all(r["busbw_GBps"] > 0 and r["world"] == 2 for r in rows)


def _local_worker(rank, world, port, stage, local, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = _cfg(stage, 2, torch.bfloat16)
    cfg.local_grad_accum = local
    eng = ZeroEngine(get_config("llama-tiny"), cfg, torch.device("cpu"), Comm())
    assert eng.local_grads == local and (eng.grad_full is not None) == local
    losses, grads0 = [], None
    for mbs in _data("llama-tiny", 2, 2 * world):
        m = eng.train_step([(t[:, :-1], t[:, 1:]) for t in mbs[2 * rank:2 * rank + 2]])
        losses.append(float(m["loss"]))
        if grads0 is None:
            grads0 = eng.full_grads()
    params = eng.full_params()
    if rank == 0:
        torch.save({"params": params, "losses": losses, "grads0": grads0}, out_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("stage", [2, 3])
def test_local_grad_accum_world2_matches_single(tmp_path, stage):
    """ZeRO-2/3 with local fp32 accumulation across GA micro-batches and ONE bf16 reduce-scatter per step
    (local_grad_accum) == single-process GA=4 training, like the per-micro-batch reduce-scatter path."""
    ref_eng = ZeroEngine(get_config("llama-tiny"), _cfg(stage, 4), torch.device("cpu"))
    ref_grads0 = None
    for mbs in _data("llama-tiny", 2, 4):
        ref_eng.train_step([(t[:, :-1], t[:, 1:]) for t in mbs])
        if ref_grads0 is None:
            ref_grads0 = ref_eng.full_grads()
    ref_params = ref_eng.full_params()
    for local in (True, False):
        out = str(tmp_path / f"l{int(local)}.pt")
        mp.spawn(_local_worker, args=(2, _free_port(), stage, local, out), nprocs=2, join=True)
        _compare(torch.load(out, weights_only=True), ref_params, ref_grads0, 2)


def _ckpt_worker(rank, world, port, save_dir, out_path):
    from distributed_llm_training_gpu_manager_amd.ckpt.checkpoint import AsyncCheckpointer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = ZeroEngine(get_config("llama-tiny"), _cfg(3, 1), torch.device("cpu"), Comm())
    t = _data("llama-tiny", 1, world)[0][rank]
    eng.train_step([(t[:, :-1], t[:, 1:])])
    ck = AsyncCheckpointer(eng, save_dir)
    ck.save(1, {"step": 1}, blocking=True)
    ck.close()
    full = eng.full_params()
    if rank == 0:
        torch.save(full, out_path)
    dist.barrier()
    dist.destroy_process_group()


def test_zero3_world2_checkpoint_offline_consolidation(tmp_path):
    """Shards written by two ZeRO-3 ranks -> ckpt/zero_to_fp32 (no process group) == gathered parameters."""
    from distributed_llm_training_gpu_manager_amd.ckpt import zero_to_fp32

    out = str(tmp_path / "full.pt")
    mp.spawn(_ckpt_worker, args=(2, _free_port(), str(tmp_path / "ck"), out), nprocs=2, join=True)
    ref = torch.load(out, weights_only=True)
    got = zero_to_fp32.consolidate(str(tmp_path / "ck"))
    assert set(got) == set(ref)
    for k, v in ref.items():
        assert torch.equal(got[k], v.float()), k


def _detail_worker(rank, world, port, stage, local):
    # TORCH_DISTRIBUTED_DEBUG=DETAIL wraps the process group: every collective first cross-checks its
    # op / shapes / dtypes across ranks, so an engine that issues collectives in a rank-dependent order
    # or with mismatched buffers fails here instead of hanging on RCCL
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      TORCH_DISTRIBUTED_DEBUG="DETAIL")
    dist.set_debug_level_from_env()  # the level is read at import; this process imported torch before the env
    dist.init_process_group("gloo", rank=rank, world_size=world)
    assert dist.get_debug_level() == dist.DebugLevel.DETAIL
    cfg = _cfg(stage, 2, torch.bfloat16)
    cfg.local_grad_accum = local
    cfg.max_live_parameters, cfg.max_reuse_distance = 0, 0  # re-gather every visit: the most collectives
    eng = ZeroEngine(get_config("llama-tiny"), cfg, torch.device("cpu"), Comm())
    for mbs in _data("llama-tiny", 2, 2 * world):
        eng.train_step([(t[:, :-1], t[:, 1:]) for t in mbs[2 * rank:2 * rank + 2]])
    eng.full_params()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("stage,local", [(1, False), (2, True), (3, False), (3, True)])
def test_collective_consistency_under_distributed_debug(stage, local):
    mp.spawn(_detail_worker, args=(2, _free_port(), stage, local), nprocs=2, join=True)


def _tcache_worker(rank, world, port, on, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = _cfg(3, 2, torch.bfloat16)
    cfg.transposed_weight_cache = on
    eng = ZeroEngine(get_config("llama-tiny"), cfg, torch.device("cpu"), Comm())
    # every gathered group is held through the step ('hbm' residency is unbounded on CPU), so every
    # group with a 2-D compute weight gets the W^T cache under ZeRO-3 as well
    assert bool(eng._tnames) == on
    assert all(eng.live_plan.held_through_step(gi) for gi in eng._tnames)
    losses = []
    for mbs in _data("llama-tiny", 3, 2 * world):
        m = eng.train_step([(t[:, :-1], t[:, 1:]) for t in mbs[2 * rank:2 * rank + 2]])
        losses.append(float(m["loss"]))
    if on:
        assert eng.memory_report()["weight_T_cache_GiB"] > 0
    params = eng.full_params()
    if rank == 0:
        torch.save({"params": params, "losses": losses}, out_path)
    dist.barrier()
    dist.destroy_process_group()


def test_zero3_world2_resident_transposed_cache_is_transparent(tmp_path):
    """ZeRO-3 on 2 ranks: dX through the W^T cache of the step-resident gathered weights (rebuilt after
    every optimizer step's all-gather) trains like dX through the gathered W."""
    res = {}
    for on in (False, True):
        out = str(tmp_path / f"t{int(on)}.pt")
        mp.spawn(_tcache_worker, args=(2, _free_port(), on, out), nprocs=2, join=True)
        res[on] = torch.load(out, weights_only=True)
    assert res[False]["losses"][0] == res[True]["losses"][0]
    for a, b in zip(res[False]["losses"], res[True]["losses"]):
        assert abs(a - b) < 1e-3 * max(1.0, abs(a))
    for k, v in res[False]["params"].items():
        d = (res[True]["params"][k] - v).abs()
        assert float(d.max()) <= 2 * 1e-2 * 3 + 1e-3, k
        assert float((d > 1e-3).float().mean()) < 0.02, k
