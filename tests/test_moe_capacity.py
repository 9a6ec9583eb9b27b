"""MoE capacity layout (ops.moe.CapacityPlan): expert rows as a static [G, C] batch for the library GEMMs plus a
grouped overflow region, dropless. Layout invariants, the HIP plan / gather kernels against the reference path,
and the MoE block / engine in capacity mode against autograd and against the other expert paths."""
import pytest
import torch

from distributed_llm_training_gpu_manager_amd.models import get_config
from distributed_llm_training_gpu_manager_amd.ops import gemm_mfma as gm
from distributed_llm_training_gpu_manager_amd.ops.moe import capacity_plan, capacity_rows, gather_rows


def _offsets(counts, device="cpu"):
    o = torch.zeros(len(counts) + 1, dtype=torch.int32)
    o[1:] = torch.tensor(counts).cumsum(0)
    return o.to(device)


@pytest.mark.parametrize("counts,C", [([5, 0, 9, 2], 4), ([3, 3, 3, 3], 4), ([0, 0, 12, 0], 4), ([1, 17, 0, 2], 8)])
def test_capacity_plan_layout(counts, C):
    R, G = sum(counts), len(counts)
    plan = capacity_plan(_offsets(counts), R, C)
    src, rmap = plan.exp_src.long(), plan.row_map
    # every sorted row lands on exactly one expanded row, and that row points back at it
    assert sorted(rmap.tolist()) == sorted(set(rmap.tolist()))
    assert torch.equal(src[rmap], torch.arange(R))
    off = 0
    ovf = 0
    for e, n in enumerate(counts):
        for r in range(n):
            x = int(rmap[off + r])
            if r < C:
                assert x == e * C + r
            else:
                assert x == G * C + ovf + (r - C)
        ovf += max(0, n - C)
        off += n
    assert plan.ovf_offsets.tolist() == [0] + list(torch.tensor([max(0, n - C) for n in counts]).cumsum(0).tolist())
    assert int(plan.nrows) == G * C + ovf
    # padding capacity rows and unused overflow rows point nowhere
    used = set(rmap.tolist())
    assert all(int(src[x]) == -1 for x in range(plan.rows) if x not in used)


def test_capacity_rows():
    assert capacity_rows(8192, 8, 1.125, 64) == 1152
    assert capacity_rows(8192, 8, 1.0, 64) == 1024
    assert capacity_rows(10, 8, 1.0, 64) == 64


@pytest.mark.gpu
@pytest.mark.parametrize("counts,C", [([5, 0, 9, 2], 4), ([700, 1300, 0, 1048], 1024), ([0] * 7 + [300], 64)])
def test_capacity_plan_and_gather_gpu_match_reference(counts, C):
    R = sum(counts)
    ref = capacity_plan(_offsets(counts), R, C)
    got = capacity_plan(_offsets(counts, "cuda"), R, C)
    assert torch.equal(got.exp_src.cpu(), ref.exp_src)
    assert torch.equal(got.row_map.cpu(), ref.row_map)
    assert torch.equal(got.ovf_offsets.cpu(), ref.ovf_offsets)
    assert int(got.nrows) == int(ref.nrows)
    T = 97
    src = torch.randn(T, 136).to(torch.bfloat16)
    tok = torch.randint(0, T, (R,))
    out = gather_rows(src.cuda(), got.exp_src, tok.cuda(), got.nrows).cpu()
    want = gather_rows(src, ref.exp_src, tok)
    n = int(ref.nrows)
    assert torch.equal(out[:n], want[:n])


def _moe_block_check(monkeypatch, factor, align, aux=0.0):
    from distributed_llm_training_gpu_manager_amd.models.common import StepContext
    from distributed_llm_training_gpu_manager_amd.models.mixtral import MixtralBlock
    from distributed_llm_training_gpu_manager_amd.models.reference import moe_ref

    monkeypatch.setattr(gm, "CAPACITY", True)
    monkeypatch.setattr(gm, "CAPACITY_FACTOR", factor)
    monkeypatch.setattr(gm, "CAPACITY_ALIGN", align)
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
    assert saved[0] == "cap"
    plan = saved[8]
    pr = {("l." + k if k == "router" else "l.experts." + k): v.clone().requires_grad_(True) for k, v in p.items()}
    xr = x.clone().requires_grad_(True)
    ref = moe_ref(xr, pr, "l.", mc)
    assert float((out - ref).abs().max()) < 1e-5
    dout = torch.randn(T, D)
    ((ref * dout).sum() * ctx.grad_scale).backward()
    g = {k: torch.zeros_like(v) for k, v in p.items()}
    dx = blk.moe_backward(p, g, x, saved, dout * ctx.grad_scale, ctx)
    assert float((dx - xr.grad).abs().max() / xr.grad.abs().max()) < 1e-5
    for k in p:
        rk = "l." + k if k == "router" else "l.experts." + k
        assert float((g[k] - pr[rk].grad).abs().max() / pr[rk].grad.abs().max()) < 1e-5, k
    return plan


@pytest.mark.parametrize("factor,align,overflow", [(2.0, 8, False), (0.5, 8, True), (1.0, 1, True)])
def test_moe_block_capacity_exact_in_fp32(monkeypatch, factor, align, overflow):
    """Capacity-layout MoE forward / backward == autograd of the plain reference, with and without rows past
    the capacity (dropless: overflow rows take the grouped path)."""
    plan = _moe_block_check(monkeypatch, factor, align)
    assert (int(plan.nrows) > plan.gc) == overflow


def _engine_grads(mc, dev, ga, defer, budget_gb=48.0):
    from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine
    g = torch.Generator().manual_seed(5)
    mbs = [(t[:, :-1], t[:, 1:]) for t in (torch.randint(0, mc.vocab_size, (2, 33), generator=g) for _ in range(ga))]
    ec = EngineConfig(zero_stage=3, micro_batch_size=2, seq_len=32, grad_accum=ga, lr=1e-3, scheduler="constant",
                      init_device="cpu", grad_clip=0.0, defer_expert_wgrad=defer, defer_wgrad_budget_gb=budget_gb)
    eng = ZeroEngine(mc, ec, torch.device(dev))
    for i, (ids, lab) in enumerate(mbs):
        eng.micro_step(ids.to(dev), lab.to(dev), first=i == 0, last=i == ga - 1)
    return {k: v.float().cpu() for k, v in eng.full_grads().items()}


@pytest.mark.parametrize("factor", [0.5, 2.0])
def test_capacity_deferred_wgrad_matches_per_micro_batch(monkeypatch, factor):
    """The deferred dW (each expert's capacity rows of all micro-batches stacked into one batched GEMM, the
    overflow rows as one segmented grouped launch) == per-micro-batch accumulation, and == the grouped path."""
    monkeypatch.setattr(gm, "CAPACITY", True)
    monkeypatch.setattr(gm, "CAPACITY_FACTOR", factor)
    monkeypatch.setattr(gm, "CAPACITY_ALIGN", 8)
    mc = get_config("mixtral-tiny", router_aux_coef=0.0)
    per_mb = _engine_grads(mc, "cpu", 3, False)
    deferred = _engine_grads(mc, "cpu", 3, True)
    monkeypatch.setattr(gm, "CAPACITY", False)
    loop = _engine_grads(mc, "cpu", 3, False)
    for k, v in per_mb.items():
        scale = v.abs().max().clamp_min(1e-8)
        assert float((deferred[k] - v).abs().max() / scale) < 1e-5, k
        assert float((loop[k] - v).abs().max() / scale) < 1e-2, k


@pytest.mark.gpu
@pytest.mark.parametrize("factor,align", [(1.125, 64), (0.5, 16)])
def test_mixtral_capacity_mode_matches_autograd_gpu(monkeypatch, factor, align):
    """Capacity mode on the GPU (batched hipBLASLt + grouped MFMA overflow + HIP plan / gather / swiglu with a
    device row count; GA 2 -> the deferred batched dW) against the fp32 autograd reference."""
    import test_engine_numerics as ten
    monkeypatch.setattr(gm, "CAPACITY", True)
    monkeypatch.setattr(gm, "CAPACITY_FACTOR", factor)
    monkeypatch.setattr(gm, "CAPACITY_ALIGN", align)
    ten._check("cuda", "mixtral-tiny", tol=1e-1)


@pytest.mark.gpu
def test_capacity_mode_hip_graph_replay_matches_eager_gpu(monkeypatch):
    """The capacity-layout MoE micro-batch loop captures into one HIP graph (no host read anywhere: the plan,
    gathers, batched GEMMs, overflow launches and the deferred batched dW are all device-driven) and trains
    like the eager loop."""
    import test_engine_numerics as ten
    monkeypatch.setattr(gm, "CAPACITY", True)
    monkeypatch.setattr(gm, "CAPACITY_ALIGN", 16)
    eg, lg = ten._train("cuda", "mixtral-tiny", True, stage=3)
    ee, le = ten._train("cuda", "mixtral-tiny", False, stage=3)
    assert eg._graph is not None and eg._graph_state == "warm", "graph was not captured"
    for a, b in zip(lg, le):
        assert abs(a - b) <= 1e-4 * max(1.0, abs(b)), (lg, le)
    err = float((eg.master - ee.master).abs().max() / ee.master.abs().max())
    assert err < 1e-4, err


@pytest.mark.parametrize("counts", [[5, 0, 9, 70], [64, 1, 0, 0], [0, 0, 0, 3]])
def test_pad_plan_and_remapped_transpose(counts):
    from distributed_llm_training_gpu_manager_amd.ops.gemm import transpose
    from distributed_llm_training_gpu_manager_amd.ops.moe import pad_plan, padded_rows
    R = sum(counts)
    src, poff = pad_plan(_offsets(counts), R, 64)
    assert src.numel() == padded_rows(R, len(counts), 64)
    assert all((b - a) % 64 == 0 for a, b in zip(poff.tolist()[:-1], poff.tolist()[1:]))
    x = torch.randn(R, 24)
    xt = transpose(x, rows=src)
    off = 0
    for e, n in enumerate(counts):
        p0 = int(poff[e])
        assert torch.equal(xt[:, p0:p0 + n], x[off:off + n].t())
        assert float(xt[:, p0 + n:int(poff[e + 1])].abs().sum()) == 0.0
        off += n


@pytest.mark.gpu
@pytest.mark.parametrize("counts", [[5, 0, 9, 70], [700, 1300, 0, 1048]])
def test_pad_plan_and_remapped_transpose_gpu(counts):
    from distributed_llm_training_gpu_manager_amd.ops.gemm import transpose
    from distributed_llm_training_gpu_manager_amd.ops.moe import pad_plan
    R = sum(counts)
    src_c, poff_c = pad_plan(_offsets(counts), R, 64)
    src_g, poff_g = pad_plan(_offsets(counts, "cuda"), R, 64)
    assert torch.equal(src_g.cpu(), src_c) and torch.equal(poff_g.cpu(), poff_c)
    x = torch.randn(R, 136).to(torch.bfloat16)
    assert torch.equal(transpose(x.cuda(), rows=src_g).cpu(), transpose(x, rows=src_c))


@pytest.mark.gpu
def test_kmajor_segmented_wgrad_gpu_matches_fp32():
    """The K-contiguous segmented grouped dW (aligned re-layout, two segments, uneven and empty experts) against
    an fp32 reference."""
    from distributed_llm_training_gpu_manager_amd.ops.gemm import transpose
    from distributed_llm_training_gpu_manager_amd.ops.moe import pad_plan
    G, M, N = 4, 256, 512
    torch.manual_seed(0)
    segs = [[130, 0, 300, 77], [5, 250, 0, 252]]  # one row count: one padded stride
    a_t, b_t, offs, ref = [], [], [], torch.zeros(G, M, N)
    for counts in segs:
        R = sum(counts)
        a = torch.randn(R, M).to(torch.bfloat16)
        b = torch.randn(R, N).to(torch.bfloat16)
        src, poff = pad_plan(_offsets(counts, "cuda"), R, 64)
        a_t.append(transpose(a.cuda(), rows=src))
        b_t.append(transpose(b.cuda(), rows=src))
        offs.append(poff)
        o = 0
        for e, n in enumerate(counts):
            ref[e] += a[o:o + n].float().t() @ b[o:o + n].float()
            o += n
    out = torch.zeros(G, M, N, device="cuda")
    gm.grouped_wgrad_segments(out, a_t, b_t, torch.stack(offs), acc=False, kmajor=True)
    err = float((out.cpu() - ref).abs().max() / ref.abs().max())
    assert err < 1e-5, err


def _multi_case(device="cpu"):
    from distributed_llm_training_gpu_manager_amd.ops.gemm import transpose_multi
    from distributed_llm_training_gpu_manager_amd.ops.moe import pad_plan_multi
    sets = [[130, 0, 300, 77], [5, 250, 0, 190], [64, 1, 2, 0]]
    offs = torch.stack([_offsets(c) for c in sets]).to(device)
    src, poff = pad_plan_multi(offs, sum(sum(c) for c in sets), 64)
    return sets, src, poff, transpose_multi


def test_pad_plan_multi_and_transpose_multi_cpu():
    sets, src, poff, transpose_multi = _multi_case()
    assert all((b - a) % 64 == 0 for a, b in zip(poff.tolist()[:-1], poff.tolist()[1:]))
    xs = [torch.randn(sum(c), 16) for c in sets]
    xt = transpose_multi(xs, src)
    for e in range(4):
        want = torch.cat([xs[t][sum(c[:e]):sum(c[:e + 1])] for t, c in enumerate(sets)]).t()
        p0, n = int(poff[e]), want.shape[1]
        assert torch.equal(xt[:, p0:p0 + n], want)
        assert float(xt[:, p0 + n:int(poff[e + 1])].abs().sum()) == 0.0


@pytest.mark.gpu
def test_kmajor_grouped_wgrad_multi_gpu_matches_fp32():
    """The deferred expert dW as ONE grouped-K launch over K-contiguous operands: several micro-batches' rows
    transposed by one launch into the aligned re-layout (uneven / empty experts), against fp32."""
    sets, src_c, poff_c, transpose_multi = _multi_case()
    _, src, poff, _ = _multi_case("cuda")
    assert torch.equal(src.cpu(), src_c) and torch.equal(poff.cpu(), poff_c)
    G, M, N = 4, 256, 512
    torch.manual_seed(1)
    a = [torch.randn(sum(c), M).to(torch.bfloat16) for c in sets]
    b = [torch.randn(sum(c), N).to(torch.bfloat16) for c in sets]
    at_ = transpose_multi([t.cuda() for t in a], src)
    bt_ = transpose_multi([t.cuda() for t in b], src)
    assert torch.equal(at_.cpu(), transpose_multi(a, src_c))
    out = torch.full((G, M, N), 7.0, device="cuda")
    gm.grouped_wgrad(out, at_, bt_, poff, acc=False, kmajor=True)
    for e in range(G):
        ref = sum(a[t][sum(c[:e]):sum(c[:e + 1])].float().t() @ b[t][sum(c[:e]):sum(c[:e + 1])].float()
                  for t, c in enumerate(sets))
        got = out[e].cpu()
        if isinstance(ref, int):
            assert float(got.abs().max()) == 0.0
        else:
            assert float((got - ref).abs().max() / ref.abs().max()) < 1e-5, e
