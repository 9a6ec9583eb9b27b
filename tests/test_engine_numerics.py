"""The hand-written unit backward + ZeRO engine against a plain fp32 autograd reference."""
import pytest
import torch

from distributed_llm_training_gpu_manager_amd.models import get_config
from distributed_llm_training_gpu_manager_amd.models.reference import gpt2_loss, llama_loss
from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine


def _engine_grads(eng: ZeroEngine):
    out = {}
    for g in eng.groups:
        full = eng.grad_shard.narrow(0, g.shard_off, g.shard_numel)
        for k, v in g.views(full).items():
            out[f"{g.name}.{k}"] = v.detach().float().cpu().clone()
    return out


def _check(device: str, model: str = "llama-tiny", tol: float = 5e-2):
    mc = get_config(model, router_aux_coef=0.0)
    ec = EngineConfig(zero_stage=3, micro_batch_size=2, seq_len=64, grad_accum=2, lr=1e-3, scheduler="constant",
                      init_device="cpu", grad_clip=0.0)
    eng = ZeroEngine(mc, ec, torch.device(device))
    if mc.n_experts:
        # separate the router logits so bf16 rounding cannot flip a token's top-k choice
        for gr in eng.groups:
            if "router" in gr.layout:
                off, shape = gr.layout["router"]
                eng.master.narrow(0, gr.shard_off + off, shape[0] * shape[1]).mul_(25.0)
        eng.sync_params_from_master()
    params = {k: v.float().cpu().clone().requires_grad_(True) for k, v in eng.full_params().items()}
    g = torch.Generator().manual_seed(3)
    toks = [torch.randint(0, mc.vocab_size, (2, 65), generator=g) for _ in range(2)]
    mbs = [(t[:, :-1].to(device), t[:, 1:].to(device)) for t in toks]
    if mc.arch == "gpt2":
        ref_loss = sum(gpt2_loss(params, mc, t[:, :-1], t[:, 1:]) for t in toks) / 2
    else:
        cos, sin = (t.cpu() for t in eng.rope)
        ref_loss = sum(llama_loss(params, mc, t[:, :-1], t[:, 1:], cos, sin) for t in toks) / 2
    ref_loss.backward()
    loss_acc = torch.zeros((), device=device)
    for i, (ids, lab) in enumerate(mbs):
        loss_acc += eng.micro_step(ids, lab, first=i == 0, last=i == 1).float()
    loss = float(loss_acc) / (2 * 2 * 64)
    assert abs(loss - float(ref_loss)) < 2e-2, (loss, float(ref_loss))
    grads = _engine_grads(eng)
    for name, p in params.items():
        ref = p.grad
        got = grads[name]
        err = float((got - ref).abs().max() / ref.abs().max().clamp_min(1e-8))
        assert err < tol, (name, err)


def test_llama_manual_backward_matches_autograd_cpu():
    _check("cpu")


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_gpt2_engine_backward_matches_autograd(device):
    # tied wte: LM-head dW (fused HIP cross-entropy dlogits) + embedding scatter-add into one segment
    _check(device, "gpt2-tiny")


def test_mixtral_manual_backward_matches_autograd_cpu():
    # bf16 end to end through router + expert GEMMs: looser than the dense model
    _check("cpu", "mixtral-tiny", tol=1e-1)


@pytest.mark.gpu
def test_mixtral_manual_backward_matches_autograd_gpu():
    _check("cuda", "mixtral-tiny", tol=1e-1)


@pytest.mark.parametrize("aux", [0.0, 0.02])
def test_moe_block_exact_in_fp32(aux):
    """The hand-written MoE forward/backward (router top-2, dispatch, experts, combine, aux loss)
    against autograd of the plain reference, in fp32 (exact up to rounding)."""
    from distributed_llm_training_gpu_manager_amd.models.common import StepContext
    from distributed_llm_training_gpu_manager_amd.models.mixtral import MixtralBlock
    from distributed_llm_training_gpu_manager_amd.models.reference import moe_ref

    torch.manual_seed(0)
    mc = get_config("mixtral-tiny", router_aux_coef=aux)
    blk = MixtralBlock(mc, 0)
    D, Fd, E = mc.d_model, mc.ffn_dim, mc.n_experts
    p = {"router": torch.randn(E, D) * 0.5, "w_gate_up": torch.randn(E, 2 * Fd, D) * 0.05,
         "w_down": torch.randn(E, D, Fd) * 0.05}
    T = 64
    x = torch.randn(T, D)
    ctx = StepContext(batch=1, seq_len=T, input_ids=None, labels=None, grad_scale=1.0 / T)
    out, saved = blk.moe_forward(p, x, ctx)
    pr = {("l." + k if k == "router" else "l.experts." + k): v.clone().requires_grad_(True) for k, v in p.items()}
    xr = x.clone().requires_grad_(True)
    ref = moe_ref(xr, pr, "l.", mc)
    assert float((out - ref).abs().max()) < 1e-5
    dout = torch.randn(T, D)
    obj = (ref * dout).sum() * ctx.grad_scale
    if aux:
        logits = xr @ pr["l.router"].t()
        probs = torch.softmax(logits, -1)
        counts = torch.bincount(logits.topk(mc.top_k, -1)[1].reshape(-1), minlength=E).float()
        obj = obj + aux * E * ((counts / T) * probs.mean(0)).sum() / mc.n_layers
    obj.backward()
    g = {k: torch.zeros_like(v) for k, v in p.items()}
    dx = blk.moe_backward(p, g, x, saved, dout * ctx.grad_scale, ctx)
    assert float((dx - xr.grad).abs().max() / xr.grad.abs().max()) < 1e-5
    for k in p:
        rk = "l." + k if k == "router" else "l.experts." + k
        assert float((g[k] - pr[rk].grad).abs().max() / pr[rk].grad.abs().max()) < 1e-5, k


@pytest.mark.gpu
def test_llama_manual_backward_matches_autograd_gpu():
    _check("cuda")


@pytest.mark.gpu
def test_engine_gpu_matches_cpu_training():
    """Same init, same data: a few optimizer steps on the GPU kernels track the CPU reference path."""
    mc = get_config("llama-tiny")
    losses = {}
    for dev in ("cpu", "cuda"):
        ec = EngineConfig(zero_stage=3, micro_batch_size=2, seq_len=128, grad_accum=1, lr=2e-3,
                          scheduler="constant", init_device="cpu")
        eng = ZeroEngine(mc, ec, torch.device(dev))
        g = torch.Generator().manual_seed(5)
        toks = torch.randint(0, mc.vocab_size, (2, 129), generator=g).to(dev)
        mb = [(toks[:, :-1].contiguous(), toks[:, 1:].contiguous())]
        losses[dev] = [float(eng.train_step(mb)["loss"]) for _ in range(4)]
    for a, b in zip(losses["cpu"], losses["cuda"]):
        assert abs(a - b) < 3e-2 * max(1.0, abs(a)), losses


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("stage", [1, 3])
def test_transposed_weight_cache_is_transparent(device, stage):
    """dX through the cached W^T (refreshed after every optimizer step) == dX through W."""
    mc = get_config("llama-tiny")
    res = {}
    for on in (False, True):
        ec = EngineConfig(zero_stage=stage, micro_batch_size=2, seq_len=32, grad_accum=2, lr=1e-2,
                          scheduler="constant", init_device="cpu", transposed_weight_cache=on)
        eng = ZeroEngine(mc, ec, torch.device(device))
        assert bool(eng._tnames) == on
        g = torch.Generator().manual_seed(9)
        losses = []
        for _ in range(3):
            mbs = []
            for _ in range(2):
                t = torch.randint(0, mc.vocab_size, (2, 33), generator=g).to(device)
                mbs.append((t[:, :-1], t[:, 1:]))
            losses.append(float(eng.train_step(mbs)["loss"]))
        if on:
            assert eng.memory_report()["weight_T_cache_GiB"] > 0
        res[on] = (losses, {k: v.float().cpu() for k, v in eng.full_params().items()})
    assert res[False][0][0] == res[True][0][0]
    for a, b in zip(res[False][0], res[True][0]):
        assert abs(a - b) < 1e-3 * max(1.0, abs(a))
    for k, v in res[False][1].items():
        d = (res[True][1][k] - v).abs()
        assert float(d.max()) <= 2 * 1e-2 * 3 + 1e-3, k
        assert float((d > 1e-3).float().mean()) < 0.02, k


def _train(device, model, graphs, steps=4, stage=0, seq=64):
    mc = get_config(model)
    ec = EngineConfig(zero_stage=stage, micro_batch_size=2, seq_len=seq, grad_accum=3, lr=1e-3,
                      scheduler="constant", init_device="cpu", hip_graphs=graphs)
    eng = ZeroEngine(mc, ec, torch.device(device))
    g = torch.Generator().manual_seed(11)
    losses = []
    for _ in range(steps):
        toks = [torch.randint(0, mc.vocab_size, (2, seq + 1), generator=g) for _ in range(3)]
        m = eng.train_step([(t[:, :-1].to(device), t[:, 1:].to(device)) for t in toks])
        losses.append(float(m["loss"]))
    return eng, losses


def test_hip_graphs_flag_is_inert_on_cpu():
    """CPU engines never capture (graph_capturable is False) and train exactly as eager."""
    e1, l1 = _train("cpu", "llama-tiny", True, steps=2)
    e2, l2 = _train("cpu", "llama-tiny", False, steps=2)
    assert not e1.graph_capturable() and e1._graph is None
    assert l1 == l2 and torch.equal(e1.master, e2.master)


@pytest.mark.gpu
@pytest.mark.parametrize("model,stage", [("llama-tiny", 0), ("gpt2-tiny", 3), ("mixtral-tiny", 3)])
def test_hip_graph_replay_matches_eager_gpu(model, stage):
    """The captured micro-batch loop (one graph replay per step, new token ids each step) trains the
    same model as the eager loop: same losses and fp32 master weights after several optimizer steps.
    Mixtral on the default grouped expert path: the capture itself proves the MoE micro-batch loop has no
    host synchronisation (a device-to-host read of the routing counts would abort it)."""
    eg, lg = _train("cuda", model, True, stage=stage)
    ee, le = _train("cuda", model, False, stage=stage)
    assert eg._graph is not None and eg._graph_state == "warm", "graph was not captured"
    for a, b in zip(lg, le):
        assert abs(a - b) <= 1e-4 * max(1.0, abs(b)), (lg, le)
    err = float((eg.master - ee.master).abs().max() / ee.master.abs().max())
    assert err < 1e-4, err


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["llama-tiny", "mixtral-tiny"])
def test_optimizer_overlap_matches_flat_update_gpu(model):
    """cfg.optimizer_overlap (one AdamW launch per group on a side stream, each waited for at the group's next
    fetch) trains the same model bit for bit as the single flat launch: losses, fp32 master, second moment and
    the bf16 compute copy after several clipped steps."""
    mc = get_config(model)
    res = {}
    for on in (False, True):
        ec = EngineConfig(zero_stage=3, micro_batch_size=2, seq_len=64, grad_accum=3, lr=1e-3, grad_clip=0.5,
                          scheduler="constant", init_device="cpu", optimizer_overlap=on)
        eng = ZeroEngine(mc, ec, torch.device("cuda"))
        g = torch.Generator().manual_seed(13)
        losses = []
        for _ in range(4):
            toks = [torch.randint(0, mc.vocab_size, (2, 65), generator=g) for _ in range(3)]
            m = eng.train_step([(t[:, :-1].cuda(), t[:, 1:].cuda()) for t in toks])
            losses.append(float(m["loss"]))
        assert (eng._opt_stream is not None) == on
        res[on] = (losses, eng.master.cpu(), eng.exp_avg_sq.cpu(), eng.p16_shard.cpu())
    assert res[True][0] == res[False][0]
    for a, b in zip(res[True][1:], res[False][1:]):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["llama-tiny", "mixtral-tiny"])
def test_side_stream_work_is_waited_for_gpu(model):
    """The W^T cache rebuild and the MoE dW re-layout run on side streams (utils.streams): with that work spun
    first, the trained state is bit-identical to a run without the spin -- every consumer waits for its event."""
    from distributed_llm_training_gpu_manager_amd.utils import streams
    mc = get_config(model)
    res = {}
    for delay in (0, 3_000_000):
        streams.TEST_DELAY_CYCLES["cycles"] = delay
        try:
            ec = EngineConfig(zero_stage=3, micro_batch_size=2, seq_len=64, grad_accum=3, lr=1e-3,
                              scheduler="constant", init_device="cpu")
            eng = ZeroEngine(mc, ec, torch.device("cuda"))
            g = torch.Generator().manual_seed(17)
            for _ in range(3):
                toks = [torch.randint(0, mc.vocab_size, (2, 65), generator=g) for _ in range(3)]
                eng.train_step([(t[:, :-1].cuda(), t[:, 1:].cuda()) for t in toks])
            res[delay] = (eng.master.cpu(), eng.exp_avg_sq.cpu())
        finally:
            streams.TEST_DELAY_CYCLES["cycles"] = 0
    for a, b in zip(res[0], res[3_000_000]):
        assert torch.equal(a, b)


@pytest.mark.gpu
def test_side_stream_inputs_survive_block_reuse_gpu(monkeypatch):
    """Side-stream ordering under allocator pressure: the MoE dW re-layout's side stream lags by ~15 ms and, right
    after every flush, the issuing stream grabs the re-layout row plan's block whenever the allocator hands it out
    again and scribbles over it; the trained state must stay bit-identical to an undisturbed run. (Round 5: with
    the plan not record_stream-ed the block did come back at once -- 6 times in this test -- and the state still
    matched, because the issuing stream waits for the side stream's event before the flush returns; the plan is
    recorded now, so that ordering no longer rests on where the join sits.)"""
    from distributed_llm_training_gpu_manager_amd.models import mixtral as mx
    from distributed_llm_training_gpu_manager_amd.utils import streams
    mc = get_config("mixtral-tiny")
    orig, orig_plan = mx.MixtralBlock._flush_wgrad_grouped, mx.pad_plan_multi
    plans, held = [], []

    def plan(offs, rows, *a, **k):
        src, poff = orig_plan(offs, rows, *a, **k)
        plans.append((src.data_ptr(), src.numel()))
        return src, poff

    def scribbled(self, g, ctx=None):
        plans.clear()
        orig(self, g, ctx)
        # take the row plan's block if the allocator hands it out again right away (it must not while the side
        # stream still reads it) and fill it with (segment 1, row 5): an in-range row, so a read of the reused
        # block gives a wrong result instead of a wild address
        for ptr, n in plans:
            for _ in range(64):
                t = torch.empty(n, dtype=torch.int32, device="cuda")
                held.append(t)
                if t.data_ptr() == ptr:
                    t.fill_((1 << 24) | 5)
                    reused.append(ptr)
                    break
    reused = []

    res = {}
    for disturb in (False, True):
        streams.TEST_DELAY_CYCLES["cycles"] = 30_000_000 if disturb else 0
        if disturb:
            monkeypatch.setattr(mx.MixtralBlock, "_flush_wgrad_grouped", scribbled)
            monkeypatch.setattr(mx, "pad_plan_multi", plan)
        try:
            ec = EngineConfig(zero_stage=3, micro_batch_size=2, seq_len=64, grad_accum=3, lr=1e-3,
                              scheduler="constant", init_device="cpu")
            eng = ZeroEngine(mc, ec, torch.device("cuda"))
            g = torch.Generator().manual_seed(17)
            for _ in range(3):
                toks = [torch.randint(0, mc.vocab_size, (2, 65), generator=g) for _ in range(3)]
                eng.train_step([(t[:, :-1].cuda(), t[:, 1:].cuda()) for t in toks])
                held.clear()
            res[disturb] = (eng.master.cpu(), eng.exp_avg_sq.cpu())
        finally:
            streams.TEST_DELAY_CYCLES["cycles"] = 0
    assert plans, "the deferred expert dW re-layout did not run"
    for a, b in zip(res[False], res[True]):
        assert torch.equal(a, b), f"state differs (row-plan blocks reused: {len(reused)})"


def test_gpt2_kept_graph_matches_activation_checkpointing_cpu():
    """GPT-2 blocks keep their forward autograd graph; with activation checkpointing the engine re-runs
    the block right before its backward instead. Both must train identically."""
    mc = get_config("gpt2-tiny")
    res = {}
    for ck in (False, True):
        ec = EngineConfig(zero_stage=3, micro_batch_size=2, seq_len=64, grad_accum=2, lr=1e-2, scheduler="constant",
                          init_device="cpu", activation_checkpointing=ck)
        eng = ZeroEngine(mc, ec, torch.device("cpu"))
        g = torch.Generator().manual_seed(1)
        losses = []
        for _ in range(3):
            mbs = []
            for _ in range(2):
                t = torch.randint(0, mc.vocab_size, (2, 65), generator=g)
                mbs.append((t[:, :-1], t[:, 1:]))
            losses.append(float(eng.train_step(mbs)["loss"]))
        res[ck] = losses
    assert res[False] == res[True], res


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("hq,hkv,d", [(4, 4, 64), (8, 2, 128)])
def test_packed_qkv_attention_matches_fp32_reference(device, hq, hkv, d):
    """flash_attention_qkv (one packed dqkv from the HIP backward) == fp32 autograd attention."""
    from distributed_llm_training_gpu_manager_amd.models.reference import _attn
    from distributed_llm_training_gpu_manager_amd.ops import flash_attention_qkv

    B, S = 2, 256
    g = torch.Generator().manual_seed(4)
    qkv32 = torch.randn(B * S, (hq + 2 * hkv) * d, generator=g)
    dout = torch.randn(B, S, hq, d, generator=g)
    x = qkv32.to(device=device, dtype=torch.bfloat16).requires_grad_(True)
    out = flash_attention_qkv(x, B, S, hq, hkv, d)
    out.backward(dout.to(device=device, dtype=torch.bfloat16))
    r = qkv32.clone().requires_grad_(True)
    f = r.view(B, S, -1)
    ref = _attn(f[..., :hq * d].unflatten(2, (hq, d)), f[..., hq * d:(hq + hkv) * d].unflatten(2, (hkv, d)),
                f[..., (hq + hkv) * d:].unflatten(2, (hkv, d)))
    ref.backward(dout)
    assert float((out.float().cpu() - ref).abs().max()) < 3e-2
    err = float((x.grad.float().cpu() - r.grad).abs().max() / r.grad.abs().max())
    assert err < 3e-2, err


@pytest.mark.parametrize("budget_gb", [48.0, 1e-6])
def test_mixtral_deferred_expert_wgrad_matches_per_micro_batch(budget_gb):
    """Expert dW over the step's concatenated micro-batches (and, with a tiny stash budget, flushed every
    micro-batch) equals the per-micro-batch accumulation."""
    mc = get_config("mixtral-tiny", router_aux_coef=0.0)
    g = torch.Generator().manual_seed(5)
    mbs = [(t[:, :-1], t[:, 1:]) for t in (torch.randint(0, mc.vocab_size, (2, 33), generator=g) for _ in range(3))]
    grads = {}
    for defer in (False, True):
        ec = EngineConfig(zero_stage=3, micro_batch_size=2, seq_len=32, grad_accum=3, lr=1e-3,
                          scheduler="constant", init_device="cpu", grad_clip=0.0, defer_expert_wgrad=defer,
                          defer_wgrad_budget_gb=budget_gb)
        eng = ZeroEngine(mc, ec, torch.device("cpu"))
        for i, (ids, lab) in enumerate(mbs):
            eng.micro_step(ids, lab, first=i == 0, last=i == 2)
        grads[defer] = _engine_grads(eng)
    for k, v in grads[False].items():
        err = float((grads[True][k] - v).abs().max() / v.abs().max().clamp_min(1e-8))
        assert err < 1e-5, (k, err)


def test_llama_head_chunked_logits_match_whole(monkeypatch):
    """A micro-batch whose [T, V] logits exceed the budget runs the LM head + cross-entropy in token chunks
    (loss in the forward, logits recomputed per chunk in the backward): same loss and gradients."""
    from distributed_llm_training_gpu_manager_amd.models.llama import LlamaHead
    mc = get_config("llama-tiny")
    g = torch.Generator().manual_seed(7)
    mbs = [(t[:, :-1], t[:, 1:]) for t in (torch.randint(0, mc.vocab_size, (2, 65), generator=g) for _ in range(2))]
    res = {}
    for chunked in (False, True):
        monkeypatch.setattr(LlamaHead, "logits_budget_bytes", 1 if chunked else 6 << 30)
        monkeypatch.setattr(LlamaHead, "chunk_tokens", 48)  # 128 tokens -> chunks of 48, 48, 32
        ec = EngineConfig(zero_stage=3, micro_batch_size=2, seq_len=64, grad_accum=2, lr=1e-3,
                          scheduler="constant", init_device="cpu", grad_clip=0.0)
        eng = ZeroEngine(mc, ec, torch.device("cpu"))
        loss = sum(float(eng.micro_step(ids, lab, first=i == 0, last=i == 1)) for i, (ids, lab) in enumerate(mbs))
        res[chunked] = (loss, _engine_grads(eng))
    assert abs(res[True][0] - res[False][0]) < 1e-4 * abs(res[False][0])
    for k, v in res[False][1].items():
        err = float((res[True][1][k] - v).abs().max() / v.abs().max().clamp_min(1e-8))
        assert err < 1e-4, (k, err)


@pytest.mark.gpu
def test_llama_chunked_head_matches_autograd_gpu(monkeypatch):
    from distributed_llm_training_gpu_manager_amd.models.llama import LlamaHead
    monkeypatch.setattr(LlamaHead, "logits_budget_bytes", 1)
    monkeypatch.setattr(LlamaHead, "chunk_tokens", 48)
    _check("cuda")


def test_mixtral_grouped_deferred_wgrad_matches_per_micro_batch_cpu(monkeypatch):
    """The grouped expert path (device offsets) with the weight gradients deferred to the step's last
    micro-batch -- one segmented grouped dW GEMM per weight over every stashed micro-batch's rows -- equals the
    per-micro-batch grouped dW. CPU run of the same code (grouped ops' reference path)."""
    from distributed_llm_training_gpu_manager_amd.models.mixtral import MixtralBlock
    from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine
    monkeypatch.setattr(MixtralBlock, "_grouped", lambda self, x: True)
    mc = get_config("mixtral-tiny")
    g = torch.Generator().manual_seed(4)
    data = [torch.randint(0, mc.vocab_size, (2, 33), generator=g) for _ in range(3)]
    grads = {}
    orig = MixtralBlock._flush_wgrad_grouped
    for dw in (False, True):
        ec = EngineConfig(zero_stage=3, micro_batch_size=2, seq_len=32, grad_accum=3, lr=1e-3, scheduler="constant",
                          init_device="cpu", defer_expert_wgrad=dw)
        eng = ZeroEngine(mc, ec, torch.device("cpu"))
        flushed = []
        monkeypatch.setattr(MixtralBlock, "_flush_wgrad_grouped",
                            lambda self, gg, ctx=None: (flushed.append(len(self._wstash)), orig(self, gg, ctx))[1])
        for i, t in enumerate(data):
            eng.micro_step(t[:, :-1], t[:, 1:], first=i == 0, last=i == 2)
        assert (flushed and flushed[0] == 3) if dw else not flushed
        grads[dw] = eng.full_grads()
    for k, v in grads[False].items():
        err = float((grads[True][k] - v).abs().max() / v.abs().max().clamp_min(1e-8))
        assert err < 1e-2, (k, err)


@pytest.mark.parametrize("ga", [1, 3])
def test_mixtral_fused_expert_grad_stats_match_grad_stats_cpu(monkeypatch, ga):
    """The expert gradients' statistics tallied by the last grouped dW launch of the step (non-deferred at
    GA 1, the K-major deferred flush at GA 3) equal ops.grad_stats over the expert groups."""
    from distributed_llm_training_gpu_manager_amd.models.mixtral import MixtralBlock
    from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine
    monkeypatch.setattr(MixtralBlock, "_grouped", lambda self, x: True)
    mc = get_config("mixtral-tiny")
    g = torch.Generator().manual_seed(5)
    data = [torch.randint(0, mc.vocab_size, (2, 33), generator=g) for _ in range(ga)]
    ec = EngineConfig(zero_stage=3, micro_batch_size=2, seq_len=32, grad_accum=ga, lr=1e-3, scheduler="constant",
                      init_device="cpu", fused_expert_grad_stats=True)
    eng = ZeroEngine(mc, ec, torch.device("cpu"))
    for i, t in enumerate(data):
        eng.micro_step(t[:, :-1], t[:, 1:], first=i == 0, last=i == ga - 1)
    fused = eng._xstats_ok
    assert fused
    eng._global_grad_stats()
    st_fused = eng.stats[:2].clone()
    eng._xstats_ok = False
    eng._global_grad_stats()
    st_ref = eng.stats[:2].clone()
    assert float(st_ref[0]) > 0 and float(st_ref[1]) == 0
    assert abs(float(st_fused[0]) - float(st_ref[0])) <= 1e-5 * float(st_ref[0])
    assert float(st_fused[1]) == 0
