"""The deferred expert dW's aligned re-layout (ops.moe.pad_plan / pad_plan_multi + the row-remapped transposes) and the
K-contiguous grouped-K / segmented dW GEMMs that consume it (csrc/kernels/moe.hip, gemm_mfma.hip)."""
import pytest
import torch

from distributed_llm_training_gpu_manager_amd.ops import gemm_mfma as gm


def _offsets(counts, device="cpu"):
    o = torch.zeros(len(counts) + 1, dtype=torch.int32)
    o[1:] = torch.tensor(counts).cumsum(0)
    return o.to(device)


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
