"""fp16 instantiations of the HIP kernels (the DeepSpeed "fp16" compute path) against the fp32 PyTorch
reference of the same op -- the bf16 versions are covered by test_kernels_gpu.py."""
import math

import pytest
import torch

from distributed_llm_training_gpu_manager_amd import ops
from distributed_llm_training_gpu_manager_amd.ops import attention as attn_ops
from distributed_llm_training_gpu_manager_amd.ops.moe import moe_combine, moe_combine_bwd

pytestmark = pytest.mark.gpu
DEV = "cuda"
H = torch.float16


def rel_err(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-6))


@pytest.mark.parametrize("D", [256, 4096])
def test_rmsnorm_fp16(D):
    torch.manual_seed(0)
    T = 45
    x, r = torch.randn(T, D, dtype=H), torch.randn(T, D, dtype=H)
    w = (1 + 0.1 * torch.randn(D)).to(H)
    y_ref, h_ref, rs_ref = ops.rmsnorm_fwd(x, w, 1e-5, residual=r)
    y, h, rs = ops.rmsnorm_fwd(x.to(DEV), w.to(DEV), 1e-5, residual=r.to(DEV))
    assert y.dtype == H and rel_err(y, y_ref) < 5e-3 and rel_err(h, h_ref) < 5e-3
    dy = torch.randn(T, D, dtype=H)
    dw_ref = torch.empty(D)
    dx_ref = ops.rmsnorm_bwd(dy, h_ref, w, rs_ref, dw_ref, dres=dy)
    dw = torch.empty(D, device=DEV)
    dx = ops.rmsnorm_bwd(dy.to(DEV), h, w.to(DEV), rs, dw, dres=dy.to(DEV))
    assert rel_err(dx, dx_ref) < 5e-3 and rel_err(dw, dw_ref) < 1e-3


def test_rope_swiglu_ce_fp16():
    torch.manual_seed(0)
    hd, S, Hh = 128, 64, 6
    cos, sin = ops.rope_tables(hd, S, 500000.0)
    qkv = torch.randn(2 * S, Hh * hd, dtype=H)
    ref = qkv.clone()
    ops.rope_(ref, cos, sin, 4, hd, S)
    g = qkv.to(DEV)
    ops.rope_(g, cos.to(DEV), sin.to(DEV), 4, hd, S)
    assert rel_err(g, ref) < 5e-3
    gu, dy = torch.randn(33, 1024, dtype=H), torch.randn(33, 512, dtype=H)
    assert rel_err(ops.swiglu_fwd(gu.to(DEV)), ops.swiglu_fwd(gu)) < 5e-3
    assert rel_err(ops.swiglu_bwd(dy.to(DEV), gu.to(DEV)), ops.swiglu_bwd(dy, gu)) < 5e-3
    logits = (3 * torch.randn(17, 32000)).to(H)
    labels = torch.randint(0, 32000, (17,))
    lr = logits.clone()
    loss_ref, lse_ref = ops.cross_entropy_fwd_bwd_(lr, labels, 1.0 / 17)
    lg = logits.to(DEV)
    loss, lse = ops.cross_entropy_fwd_bwd_(lg, labels.to(DEV), 1.0 / 17)
    assert rel_err(lse, lse_ref) < 1e-4 and rel_err(lg, lr) < 1e-2


@pytest.mark.parametrize("B,S,Hq,Hkv,D", [(1, 256, 8, 2, 128), (2, 200, 4, 2, 64), (1, 1024, 4, 4, 128)])
def test_flash_attention_fp16(B, S, Hq, Hkv, D):
    torch.manual_seed(0)
    q = torch.randn(B, S, Hq, D, dtype=H)
    k = torch.randn(B, S, Hkv, D, dtype=H)
    v = torch.randn(B, S, Hkv, D, dtype=H)
    do = torch.randn(B, S, Hq, D, dtype=H)
    scale = 1 / math.sqrt(D)
    o_ref, lse_ref = attn_ops._ref_fwd(q, k, v, scale, True)
    o, lse = ops.flash_attn_fwd(q.to(DEV), k.to(DEV), v.to(DEV), scale, True)
    assert o.dtype == H and rel_err(o, o_ref) < 1e-2 and rel_err(lse, lse_ref) < 1e-3
    dq_ref, dk_ref, dv_ref = attn_ops._ref_bwd(do, q, k, v, o_ref, lse_ref, scale, True)
    dq, dk, dv = ops.flash_attn_bwd(do.to(DEV), q.to(DEV), k.to(DEV), v.to(DEV), o, lse, scale, True)
    assert rel_err(dq, dq_ref) < 2e-2 and rel_err(dk, dk_ref) < 2e-2 and rel_err(dv, dv_ref) < 2e-2


def test_optimizer_accumulate_moe_fp16():
    torch.manual_seed(0)
    n = 100_003
    p, gr = torch.randn(n), torch.randn(n)
    m, v = torch.zeros(n), torch.zeros(n)
    kw = dict(lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.01, step=1, max_norm=0.0)
    pr, mr, vr = p.clone(), m.clone(), v.clone()
    ops.adamw_step_(pr, mr, vr, gr, None, None, **kw)
    pg = p.to(DEV)
    p16 = torch.empty(n, dtype=H, device=DEV)
    ops.adamw_step_(pg, m.to(DEV), v.to(DEV), gr.to(DEV, H), p16, None, **kw)  # fp16 gradient, fp16 copy
    assert rel_err(pg, pr) < 1e-3 and rel_err(p16, pr) < 1e-3
    dst = torch.ones(4099, device=DEV)
    src = torch.randn(4099, dtype=H, device=DEV)
    ops.accumulate_(dst, src, 0.5, 1.0)
    assert rel_err(dst, 1 + 0.5 * src.float()) < 1e-6
    out = torch.empty(4099, dtype=H, device=DEV)
    ops.cast_f32_bf16_(out, dst)
    assert torch.equal(out, dst.half())
    st = torch.zeros(2, device=DEV)
    ops.grad_stats([src], st)
    assert abs(float(st[0]) - float(src.float().pow(2).sum())) / float(st[0]) < 1e-3
    T, K, D = 50, 2, 512
    y = torch.randn(T * K, D, dtype=H)
    pos = torch.randperm(T * K).view(T, K)
    gates = torch.softmax(torch.randn(T, K), -1)
    assert rel_err(moe_combine(y.to(DEV), pos.to(DEV), gates.to(DEV)), moe_combine(y, pos, gates)) < 5e-3
    dout = torch.randn(T, D, dtype=H)
    dy_ref, dg_ref = moe_combine_bwd(dout, y, pos, gates)
    dy, dg = moe_combine_bwd(dout.to(DEV), y.to(DEV), pos.to(DEV), gates.to(DEV))
    assert rel_err(dy, dy_ref) < 5e-3 and rel_err(dg, dg_ref) < 1e-3
