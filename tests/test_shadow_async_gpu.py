"""RCCL stream ordering, rehearsed on ONE MI355X.

gloo (host-staged, blocking) and the synchronous shadow rank cannot show a compute-stream / comm-stream
race. ``ShadowComm(async_mode=True)`` runs every collective the way ProcessGroupNCCL runs an RCCL one: on
the communicator's own HIP stream, ordered after the issuing stream's queued work, inputs/outputs
``record_stream``-ed, completion awaited by ``Handle.wait()`` on the consumer stream -- and it first spins
that stream for ``delay_cycles``, so a missing wait or an early overwrite corrupts the result every run.
The engine must then produce BIT-IDENTICAL optimizer state and gradients to the synchronous shadow run,
over the ZeRO stages / residency / gradient-accumulation / parameter-offload paths and the MoE
expert-parallel path (reference: ``overlap_comm: True``, /root/reference/ai_engine/deepspeed_launcher.py:137).
"""
import pytest
import torch

from distributed_llm_training_gpu_manager_amd.models import get_config
from distributed_llm_training_gpu_manager_amd.parallel.comm import ShadowComm
from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine

pytestmark = pytest.mark.gpu

STATE = ("master", "exp_avg", "exp_avg_sq", "grad_shard", "p16_shard")


def _run(model, world, async_mode, steps=3, ga=2, opt_delay=0, **kw):
    dev = torch.device("cuda", 0)
    mc = get_config(model)
    ec = EngineConfig(micro_batch_size=2, seq_len=64, grad_accum=ga, lr=1e-3, scheduler="constant", grad_clip=1.0)
    for k, v in kw.items():
        setattr(ec, k, v)
    comm = ShadowComm(world, 0, async_mode=async_mode, delay_cycles=200_000 if async_mode else 0)
    eng = ZeroEngine(mc, ec, dev, comm)
    eng._opt_delay_cycles = opt_delay
    g = torch.Generator().manual_seed(3)
    for _ in range(steps):
        mbs = []
        for _ in range(ga):
            t = torch.randint(0, mc.vocab_size, (2, 65), generator=g).to(dev)
            mbs.append((t[:, :-1].contiguous(), t[:, 1:].contiguous()))
        eng.train_step(mbs)
    torch.cuda.synchronize()
    issued = comm.issued + sum(getattr(c, "issued", 0) for c in {id(x): x for x in _comms(eng)}.values()
                               if c is not comm)
    issued += eng.mesh.issued if eng.mesh is not None else 0  # collectives the xGMI mesh ran on its streams
    out = {k: getattr(eng, k).detach().cpu().clone() for k in STATE}
    out["_layout"] = [(g.idx, g.shard_off, g.shard_numel, [sp.name for sp in g.specs]) for g in eng.groups]
    return out, issued


def _where(ref, got, k):
    """Which parameter groups the differing elements of state `k` fall in (the shard-flat layout of the run)."""
    bad = (ref[k] != got[k]).nonzero().flatten().tolist()
    hit = {}
    for i in bad:
        for gi, off, n, names in ref["_layout"]:
            if off <= i < off + n:
                hit.setdefault(gi, [names[:3], 0])[1] += 1
    return {"n_bad": len(bad), "first": bad[:4], "max_abs": float((ref[k].float() - got[k].float()).abs().max()),
            "groups": hit}


def _comms(eng):
    out = [eng.comm]
    for name in ("gather_comm", "ep_comm", "edp_comm"):
        c = getattr(eng, name, None)
        if c is not None:
            out.append(c)
    for grp in eng.groups:
        out += [c for c in (grp.comm, getattr(grp, "gcomm", None)) if c is not None]
    return out


CASES = {
    "zero2": dict(zero_stage=2, local_grad_accum=False),
    "zero2_local": dict(zero_stage=2, local_grad_accum=True),
    "zero3_resident": dict(zero_stage=3, local_grad_accum=False),
    "zero3_resident_local": dict(zero_stage=3, local_grad_accum=True),
    "zero3_nonresident": dict(zero_stage=3, max_live_parameters=0, max_reuse_distance=0, local_grad_accum=False),
    "zero3_nonresident_local": dict(zero_stage=3, max_live_parameters=0, max_reuse_distance=0,
                                    local_grad_accum=True),
    "zero3_offload_param": dict(zero_stage=3, offload_param="cpu", local_grad_accum=False),
    # the device-driven xGMI mesh transport in shadow mode (parallel/xgmi_mesh.py): gathers pulled and gradients
    # push-reduced on the mesh's own streams after the spin, versus inline on the compute stream
    "zero2_mesh": dict(zero_stage=2, local_grad_accum=False, xgmi_mesh="on"),
    "zero2_local_mesh": dict(zero_stage=2, local_grad_accum=True, xgmi_mesh="on"),
    "zero3_resident_mesh": dict(zero_stage=3, local_grad_accum=False, xgmi_mesh="on"),
    "zero3_resident_local_mesh": dict(zero_stage=3, local_grad_accum=True, xgmi_mesh="on"),
    "zero3_nonresident_mesh": dict(zero_stage=3, max_live_parameters=0, max_reuse_distance=0, local_grad_accum=False,
                                   xgmi_mesh="on"),
    "zero3_nonresident_local_mesh": dict(zero_stage=3, max_live_parameters=0, max_reuse_distance=0,
                                         local_grad_accum=True, xgmi_mesh="on"),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_async_shadow_is_bit_identical_llama(case):
    ref, n_sync = _run("llama-tiny", 4, False, **CASES[case])
    got, n_async = _run("llama-tiny", 4, True, **CASES[case])
    assert n_sync == 0 and n_async > 0  # the async run really went through the comm streams
    bad = [k for k in STATE if not torch.equal(ref[k], got[k])]
    if bad:  # say where, and whether the synchronous reference itself repeats (a race vs a nondeterministic op)
        ref2, _ = _run("llama-tiny", 4, False, **CASES[case])
        got2, _ = _run("llama-tiny", 4, True, **CASES[case])
        same = lambda a, b: all(torch.equal(a[k], b[k]) for k in STATE)  # noqa: E731
        raise AssertionError((case, {k: _where(ref, got, k) for k in bad},
                              {"ref==ref2": same(ref, ref2), "got==got2": same(got, got2),
                               "got2==ref2": same(got2, ref2), "got==ref2": same(got, ref2)}))


@pytest.mark.parametrize("stage,mesh", [(2, "off"), (3, "off"), (2, "on"), (3, "on")])
def test_async_shadow_is_bit_identical_mixtral_ep4(stage, mesh):
    kw = dict(zero_stage=stage, expert_parallel_size=4, local_grad_accum=False, xgmi_mesh=mesh)
    ref, _ = _run("mixtral-tiny", 4, False, **kw)
    got, n_async = _run("mixtral-tiny", 4, True, **kw)
    assert n_async > 0
    for k in STATE:
        assert torch.equal(ref[k], got[k]), (stage, k, float((ref[k].float() - got[k].float()).abs().max()))


@pytest.mark.parametrize("model,world,kw", [
    ("llama-tiny", 1, dict(zero_stage=3)),
    ("llama-tiny", 4, dict(zero_stage=3, local_grad_accum=True)),
    ("llama-tiny", 4, dict(zero_stage=3, max_live_parameters=0, max_reuse_distance=0, local_grad_accum=False)),
    ("mixtral-tiny", 4, dict(zero_stage=3, expert_parallel_size=4, local_grad_accum=False)),
])
def test_overlapped_optimizer_waits_per_group(model, world, kw):
    """cfg.optimizer_overlap with the optimizer stream spun before its updates (so a gather, fetch or gradient write
    that does not wait for its group's update reads or clobbers stale state): bit-identical to the flat update on the
    compute stream, with asynchronous (RCCL-ordered) collectives."""
    ref, _ = _run(model, world, True, optimizer_overlap=False, **kw)
    got, _ = _run(model, world, True, opt_delay=2_000_000, optimizer_overlap=True, **kw)
    bad = [k for k in STATE if not torch.equal(ref[k], got[k])]
    if bad:  # say where: the differing elements, and whether the reference itself repeats
        ref2, _ = _run(model, world, True, optimizer_overlap=False, **kw)
        where = {k: (int((ref[k] != got[k]).sum()), (ref[k] != got[k]).nonzero()[:4].flatten().tolist(),
                     float((ref[k].float() - got[k].float()).abs().max())) for k in bad}
        got2, _ = _run(model, world, True, opt_delay=2_000_000, optimizer_overlap=True, **kw)
        same = lambda a, b: all(torch.equal(a[k], b[k]) for k in STATE)  # noqa: E731
        raise AssertionError((model, kw, where, {"ref==ref2": same(ref, ref2), "got==ref2": same(got, ref2),
                                                 "got2==ref2": same(got2, ref2), "got2==got": same(got2, got)}))
