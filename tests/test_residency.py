"""ZeRO-3 gathered-parameter residency (stage3_max_live_parameters / stage3_max_reuse_distance).

The plan only decides WHEN a unit is all-gathered, never what it computes: a run that keeps
everything resident must match a run that re-gathers every visit bit for bit, while issuing
one all-gather per unit per optimizer step instead of two per micro-batch.
"""
import math
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_llm_training_gpu_manager_amd.models import get_config
from distributed_llm_training_gpu_manager_amd.parallel.comm import Comm
from distributed_llm_training_gpu_manager_amd.parallel.residency import ResidencyPlan, resolve_limit
from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine


def _visits(groups_per_stage):
    return list(groups_per_stage) + list(reversed(groups_per_stage))


def test_plan_counts_gathers():
    stages = [(0,), (1,), (2,), (3,)]
    sizes, gathered = [10, 20, 20, 10], [True] * 4
    v = _visits(stages)
    everything = ResidencyPlan(v, sizes, gathered, math.inf, math.inf)
    assert everything.gathers_per_step(4) == 4 and everything.resident_params == 60
    nothing = ResidencyPlan(v, sizes, gathered, 0, 0)
    assert nothing.gathers_per_step(4) == 4 * 8
    # DeepSpeed-style small budget: only the head (distance 0 from its forward to its backward) fits
    head_only = ResidencyPlan(v, sizes, gathered, 10, 0)
    assert head_only.resident_groups == [3]
    assert head_only.gathers_per_step(4) == 4 * 7
    # nothing survives the optimizer step: the last micro-batch drops the wrap-around keeps
    assert not everything.keep(7, 0, last_micro=True) and everything.keep(7, 0, last_micro=False)


def test_plan_reuse_distance_and_tied_groups():
    # GPT-2 style: group 0 (tied embedding / head) visited first and last
    stages = [(0,), (1,), (2,), (0,)]
    sizes, gathered = [50, 10, 10, 50], [True, True, True, False]
    p = ResidencyPlan(_visits(stages), sizes, gathered, math.inf, 20)
    # fwd of group 0 at v=0 -> next use at v=3 after groups 1, 2 (20 params): kept
    assert p.distance[(0, 0)] == 20 and p.keep(0, 0, last_micro=False)
    # group 1 fwd (v=1) -> its backward (v=6) after groups 2, 0, 0, 2 are fetched: 120 > 20, dropped
    assert p.distance[(1, 1)] == 10 + 50 + 50 + 10
    assert not p.keep(1, 1, last_micro=False)


def test_resolve_limit():
    assert resolve_limit(1e9, lambda: 5.0) == 1e9
    assert resolve_limit("hbm", lambda: 5.0) == 5.0
    assert resolve_limit("hbm", lambda: 5.0, unbounded_for_hbm=True) == math.inf


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mc = get_config("llama-tiny")
    g = torch.Generator().manual_seed(17 + rank)
    data = [[torch.randint(0, mc.vocab_size, (2, 33), generator=g) for _ in range(3)] for _ in range(2)]
    res = {}
    for name, live in (("regather", 0), ("resident", "hbm")):
        ec = EngineConfig(zero_stage=3, micro_batch_size=2, seq_len=32, grad_accum=3, lr=1e-2, scheduler="constant",
                          init_device="cpu", grad_clip=1.0, comm_dtype=torch.float32, max_live_parameters=live,
                          max_reuse_distance=live)
        eng = ZeroEngine(mc, ec, torch.device("cpu"), Comm())
        calls = [0]
        orig = eng.gather_comm.all_gather

        def counted(out, inp, async_op=True, _orig=orig):
            calls[0] += 1
            return _orig(out, inp, async_op=async_op)

        eng.gather_comm.all_gather = counted
        losses = [float(eng.train_step([(t[:, :-1], t[:, 1:]) for t in step])["loss"]) for step in data]
        res[name] = {"losses": losses, "params": eng.full_params(), "gathers": calls[0],
                     "planned": eng.live_plan.gathers_per_step(3) * len(data), "units": len(eng.groups)}
    if rank == 0:
        torch.save(res, out_path)
    dist.barrier()
    dist.destroy_process_group()


def test_zero3_resident_params_world2_bitwise_and_fewer_gathers(tmp_path):
    out = str(tmp_path / "r.pt")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    res = torch.load(out, weights_only=True)
    a, b = res["regather"], res["resident"]
    assert a["losses"] == b["losses"]
    for k, v in a["params"].items():
        assert torch.equal(v, b["params"][k]), k
    units, steps, ga = a["units"], 2, 3
    assert b["gathers"] == b["planned"] == units * steps  # one all-gather per unit per optimizer step
    assert a["gathers"] == a["planned"] == units * 2 * ga * steps  # forward + backward, every micro-batch
