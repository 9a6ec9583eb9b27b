"""Hand-written MFMA GEMM (csrc/kernels/gemm_mfma.hip) vs an fp32 PyTorch reference: every operand
layout, the three epilogues, and the expert-grouped modes with device-side offsets (uneven and empty
groups)."""
import pytest
import torch

from distributed_llm_training_gpu_manager_amd.ops import gemm_mfma as gm

pytestmark = pytest.mark.gpu
dev = "cuda"


def _op(shape, kmaj_rows, g):
    """A [R, C] logical operand stored either row-major or as the transpose view of a row-major tensor."""
    R, C = shape
    if kmaj_rows:
        return torch.randn(R, C, device=dev, generator=g).to(torch.bfloat16)
    return torch.randn(C, R, device=dev, generator=g).to(torch.bfloat16).t()


def _rel(x, ref):
    return float((x.float() - ref).abs().max() / ref.abs().max().clamp_min(1e-6))


@pytest.mark.parametrize("a_rowmajor", [True, False])
@pytest.mark.parametrize("b_rowmajor", [True, False])
@pytest.mark.parametrize("epi", ["bf16", "f32", "acc"])
@pytest.mark.parametrize("K", [64, 128, 320])
def test_dense_layouts_and_epilogues(a_rowmajor, b_rowmajor, epi, K):
    """K 64 / 128 / 320 = one, two (no steady state) and five K-tiles."""
    g = torch.Generator(device=dev).manual_seed(0)
    M, N = 512, 768
    a = _op((M, K), a_rowmajor, g)
    b = _op((K, N), b_rowmajor, g)
    ref = a.float() @ b.float()
    if epi == "bf16":
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        gm.mfma_mm(out, a, b)
        assert _rel(out, ref) < 1e-2
    elif epi == "f32":
        out = torch.full((M, N), 7.0, device=dev)
        gm.mfma_mm(out, a, b)
        assert _rel(out, ref) < 1e-5
    else:
        base = torch.randn(M, N, device=dev, generator=g)
        out = base.clone()
        gm.mfma_mm(out, a, b, acc=True)
        assert _rel(out, ref + base) < 1e-5


def test_weight_gradient_shape_accumulates_into_fp32():
    """dW = dy^T x with both operands token-major (the engine's layout), beta = 1, M/N tails in K."""
    g = torch.Generator(device=dev).manual_seed(1)
    T, O, I = 1024, 768, 512
    dy = torch.randn(T, O, device=dev, generator=g).to(torch.bfloat16)
    x = torch.randn(T, I, device=dev, generator=g).to(torch.bfloat16)
    w = torch.randn(O, I, device=dev, generator=g)
    ref = w + dy.float().t() @ x.float()
    assert gm.supported(w, dy.t(), x)
    gm.mfma_mm(w, dy.t(), x, acc=True)
    assert _rel(w, ref) < 1e-5


def test_grouped_rows_forward_uneven_and_empty_groups():
    g = torch.Generator(device=dev).manual_seed(2)
    sizes = [300, 0, 1, 513, 256, 77]
    R, K, N, G = sum(sizes), 512, 512, len(sizes)
    offs = torch.tensor([0] + list(torch.tensor(sizes).cumsum(0)), dtype=torch.int32, device=dev)
    x = torch.randn(R, K, device=dev, generator=g).to(torch.bfloat16)
    w = torch.randn(G, N, K, device=dev, generator=g).to(torch.bfloat16)
    out = gm.grouped_mm(x, w, offs)
    lo = 0
    for e, n in enumerate(sizes):
        if n:
            ref = x[lo:lo + n].float() @ w[e].float().t()
            assert _rel(out[lo:lo + n], ref) < 1e-2, e
        lo += n
    # [G, K, N] weights (input-gradient orientation: dy @ W)
    w2 = torch.randn(G, K, N, device=dev, generator=g).to(torch.bfloat16)
    out2 = gm.grouped_mm(x, w2, offs, transpose_w=False)
    lo = 0
    for e, n in enumerate(sizes):
        if n:
            assert _rel(out2[lo:lo + n], x[lo:lo + n].float() @ w2[e].float()) < 1e-2, e
        lo += n


@pytest.mark.parametrize("transpose_w", [True, False])
def test_grouped_dx_fused_swiglu_bwd_matches_unfused(transpose_w, monkeypatch):
    """The down projection's input gradient with the SwiGLU backward in the epilogue is bit-exact with the unfused
    pair (grouped_mm -> swiglu_bwd kernel): same bf16 rounding of dA, same fp32 math; uneven, empty, single-row and
    partial-tile groups. Also within bf16 tolerance of the fp32 PyTorch reference. (K < 4096: neither launch takes
    the tail split, which the fused launch never does.)"""
    g = torch.Generator(device=dev).manual_seed(11)
    sizes = [300, 0, 1, 513, 256, 77]
    R, K, F, G = sum(sizes), 512, 768, len(sizes)
    offs = torch.tensor([0] + list(torch.tensor(sizes).cumsum(0)), dtype=torch.int32, device=dev)
    dy = torch.randn(R, K, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(G, F, K, device=dev, generator=g) if transpose_w else
         torch.randn(G, K, F, device=dev, generator=g)).to(torch.bfloat16) * 0.1
    gu = torch.randn(R, 2 * F, device=dev, generator=g).to(torch.bfloat16)
    monkeypatch.setenv("DLGM_MOE_FUSED_SWIGLU", "1")
    got = gm.grouped_dx_swiglu(dy, w, offs, gu, transpose_w=transpose_w)
    monkeypatch.setenv("DLGM_MOE_FUSED_SWIGLU", "0")
    ref = gm.grouped_dx_swiglu(dy, w, offs, gu, transpose_w=transpose_w)
    assert got.shape == gu.shape and got.dtype == torch.bfloat16
    assert torch.equal(got.view(torch.int16), ref.view(torch.int16))
    lo = 0
    for e, n in enumerate(sizes):
        if n:
            we = w[e].float().t() if transpose_w else w[e].float()
            d = dy[lo:lo + n].float() @ we
            gg, uu = gu[lo:lo + n, :F].float(), gu[lo:lo + n, F:].float()
            s = torch.sigmoid(gg)
            want = torch.cat([d * uu * (s + gg * s * (1 - s)), d * gg * s], dim=1)
            assert _rel(got[lo:lo + n], want) < 2e-2, e
        lo += n


@pytest.mark.parametrize("transpose_w", [True, False])
def test_grouped_rows_narrow_long_k_split_k(transpose_w):
    """Narrow output (<= 16 column tiles) with a long K: 32 tiles, i.e. a single short round on every XCD, so the
    tail split runs every tile as four K parts (fp32 partials + the tail reduce); uneven / empty / single-row
    groups; also the balanced XCD remap over the real tiles."""
    g = torch.Generator(device=dev).manual_seed(7)
    sizes = [700, 0, 1, 513, 1300, 77, 256, 33]
    R, K, N, G = sum(sizes), 16384, 512, len(sizes)
    offs = torch.tensor([0] + list(torch.tensor(sizes).cumsum(0)), dtype=torch.int32, device=dev)
    x = torch.randn(R, K, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(G, N, K, device=dev, generator=g) if transpose_w else
         torch.randn(G, K, N, device=dev, generator=g)).to(torch.bfloat16)
    out = gm.grouped_mm(x, w, offs, transpose_w=transpose_w)
    lo = 0
    for e, n in enumerate(sizes):
        if n:
            we = w[e].float().t() if transpose_w else w[e].float()
            assert _rel(out[lo:lo + n], x[lo:lo + n].float() @ we) < 1e-2, e
        lo += n


@pytest.mark.parametrize("sizes,N", [
    ([1500, 0, 1, 2100, 700, 1800, 1200, 891], 4096),     # 36 row tiles x 16 = 576: 72 per XCD -> 2 rounds + 8 in 4 parts
    ([2560, 2561, 0, 2048, 1280, 1287, 768, 100], 4096),  # 44 row tiles: 88 per XCD -> a tail of 24 in 4 parts
    ([2560, 2561, 0, 2048, 1280, 1287, 768, 356], 4096),  # 45 row tiles: 90 per XCD -> a tail of 26, unsplit
    ([1500, 0, 1, 2100, 700, 1800, 1200, 891], 6144),     # 36 x 24 = 864: 108 per XCD -> 3 rounds + 12 in halves
])
@pytest.mark.parametrize("transpose_w", [True, False])
def test_grouped_rows_tail_split(sizes, N, transpose_w):
    """Grouped-M launches at the Mixtral down-projection shape (N = 4096, K = 4096) and a wider one: each XCD's whole
    rounds of tiles store bf16 directly, its short last round runs as 2-4 K parts per tile whose fp32 partials the
    tail reduce sums (the tiles on both sides of that split, partial row tiles and an empty group included)."""
    g = torch.Generator(device=dev).manual_seed(13)
    R, K, G = sum(sizes), 4096, len(sizes)
    offs = torch.tensor([0] + list(torch.tensor(sizes).cumsum(0)), dtype=torch.int32, device=dev)
    x = torch.randn(R, K, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(G, N, K, device=dev, generator=g) if transpose_w else
         torch.randn(G, K, N, device=dev, generator=g)).to(torch.bfloat16)
    out = gm.grouped_mm(x, w, offs, transpose_w=transpose_w)
    lo = 0
    for e, n in enumerate(sizes):
        if n:
            we = w[e].float().t() if transpose_w else w[e].float()
            assert _rel(out[lo:lo + n], x[lo:lo + n].float() @ we) < 1e-2, e
        lo += n


def test_grouped_rows_tail_split_is_deterministic():
    """The tail split's partials are summed in a fixed order: two launches over the same operands and routing are
    bit-identical (the engine's bit-identity checks rely on it)."""
    g = torch.Generator(device=dev).manual_seed(21)
    sizes = [1500, 0, 1, 2100, 700, 1800, 1200, 891]  # a tail of 8 tiles per XCD in 4 K parts
    R, K, N, G = sum(sizes), 4096, 4096, len(sizes)
    offs = torch.tensor([0] + list(torch.tensor(sizes).cumsum(0)), dtype=torch.int32, device=dev)
    x = torch.randn(R, K, device=dev, generator=g).to(torch.bfloat16)
    w = torch.randn(G, N, K, device=dev, generator=g).to(torch.bfloat16)
    a = gm.grouped_mm(x, w, offs)
    b = gm.grouped_mm(x, w, offs)
    assert torch.equal(a.view(torch.int16), b.view(torch.int16))


def test_grouped_weight_gradient_uneven_and_empty_groups():
    g = torch.Generator(device=dev).manual_seed(3)
    sizes = [130, 0, 700, 1]
    R, M, N, G = sum(sizes), 512, 256, len(sizes)
    offs = torch.tensor([0] + list(torch.tensor(sizes).cumsum(0)), dtype=torch.int32, device=dev)
    dy = torch.randn(R, M, device=dev, generator=g).to(torch.bfloat16)
    x = torch.randn(R, N, device=dev, generator=g).to(torch.bfloat16)
    out = torch.full((G, M, N), 3.0, device=dev)
    gm.grouped_wgrad(out, dy, x, offs)
    acc = torch.randn(G, M, N, device=dev, generator=g)
    out2 = acc.clone()
    gm.grouped_wgrad(out2, dy, x, offs, acc=True)
    lo = 0
    for e, n in enumerate(sizes):
        ref = dy[lo:lo + n].float().t() @ x[lo:lo + n].float()
        if n == 0:
            assert float(out[e].abs().max()) == 0.0
            assert torch.equal(out2[e], acc[e])
        else:
            assert _rel(out[e], ref) < 1e-5, e
            assert _rel(out2[e], ref + acc[e]) < 1e-5, e
        lo += n


def _stats_ref(t):
    fin = torch.isfinite(t)
    return float(torch.where(fin, t, torch.zeros_like(t)).double().square().sum()), float((~fin).sum())


@pytest.mark.parametrize("acc", [False, True])
@pytest.mark.parametrize("kmajor", [False, True])
def test_grouped_weight_gradient_fused_statistics(acc, kmajor):
    """The grouped-K epilogue's per-tile statistics of the stored gradient (sum of squares of the finite, count of
    the non-finite) summed = the same statistics of the whole output: uneven / empty groups, a partial M tile (K-major),
    token-major and K-major operands (spare blocks of the chunked XCD remap must not write partials), a
    non-finite accumulated value counted once."""
    g = torch.Generator(device=dev).manual_seed(11)
    sizes = [192, 0, 704, 64, 64] if kmajor else [130, 0, 700, 1, 64]
    R, M, N, G = sum(sizes), 384 if kmajor else 512, 512, len(sizes)  # partial M tile: K-contiguous rows only
    offs = torch.tensor([0] + list(torch.tensor(sizes).cumsum(0)), dtype=torch.int32, device=dev)
    dy = torch.randn(R, M, device=dev, generator=g).to(torch.bfloat16)
    x = torch.randn(R, N, device=dev, generator=g).to(torch.bfloat16)
    out = torch.randn(G, M, N, device=dev, generator=g) if acc else torch.full((G, M, N), 3.0, device=dev)
    if acc:
        out[1, 5, 7] = float("inf")  # empty group: the old value is still counted
        out[2, 300, 9] = float("nan")
    ref = out.clone() if acc else torch.zeros_like(out)
    lo = 0
    for e, n in enumerate(sizes):
        ref[e] += dy[lo:lo + n].float().t() @ x[lo:lo + n].float()
        lo += n
    st = torch.tensor([1.0, 0.0], device=dev)  # accumulated into, not overwritten
    if kmajor:
        gm.grouped_wgrad(out, dy.t().contiguous(), x.t().contiguous(), offs, acc=acc, kmajor=True, stats=st)
    else:
        gm.grouped_wgrad(out, dy, x, offs, acc=acc, stats=st)
    fin = torch.isfinite(ref)
    assert torch.equal(fin, torch.isfinite(out))
    assert _rel(torch.where(fin, out, 0.0), torch.where(fin, ref, 0.0)) < 1e-5
    ss, bad = _stats_ref(out)
    assert float(st[1]) == bad == (2.0 if acc else 0.0)
    assert abs(float(st[0]) - 1.0 - ss) <= 1e-5 * ss


@pytest.mark.parametrize("nseg", [1, 3, 8])
def test_grouped_weight_gradient_over_segments(nseg):
    """Segmented grouped-K (the deferred expert dW over a step's micro-batches): every group reduces over its
    rows of all segments; segments route differently (uneven, empty groups, a segment with no rows for a
    group, partial K tiles at every segment end); store and accumulate epilogues."""
    g = torch.Generator(device=dev).manual_seed(4 + nseg)
    G, M, N = 4, 256, 512
    segs = []
    for s in range(nseg):
        sizes = [int(x) for x in torch.randint(0, 200, (G,), generator=torch.Generator().manual_seed(s))]
        sizes[s % G] = 0  # a group with no rows in this segment
        R = sum(sizes)
        offs = [0] + list(torch.tensor(sizes).cumsum(0).tolist())
        segs.append((torch.randn(R, M, device=dev, generator=g).to(torch.bfloat16),
                     torch.randn(R, N, device=dev, generator=g).to(torch.bfloat16), offs))
    offsets = torch.tensor([o for *_, o in segs], dtype=torch.int32, device=dev)
    ref = torch.zeros(G, M, N, device=dev)
    for a, b, o in segs:
        for e in range(G):
            ref[e] += a[o[e]:o[e + 1]].float().t() @ b[o[e]:o[e + 1]].float()
    out = torch.full((G, M, N), 5.0, device=dev)
    gm.grouped_wgrad_segments(out, [s[0] for s in segs], [s[1] for s in segs], offsets)
    assert _rel(out, ref) < 1e-5
    base = torch.randn(G, M, N, device=dev, generator=g)
    out2 = base.clone()
    gm.grouped_wgrad_segments(out2, [s[0] for s in segs], [s[1] for s in segs], offsets, acc=True)
    assert _rel(out2, ref + base) < 1e-5


def test_grouped_forward_reads_nothing_on_the_host(monkeypatch):
    """The grouped MFMA expert GEMM takes the routing offsets on the device only: run it inside a HIP graph
    capture (which fails on any synchronising call) with offsets that differ from the warm-up call.
    (torch._grouped_mm is not capture-safe on this stack -- "operation not permitted when stream is
    capturing" -- so it is not a sync-free alternative.)"""
    g = torch.Generator(device=dev).manual_seed(5)
    R, K, N, G = 1024, 512, 768, 8
    x = torch.randn(R, K, device=dev, generator=g).to(torch.bfloat16)
    w = torch.randn(G, N, K, device=dev, generator=g).to(torch.bfloat16)
    offs = torch.tensor([0, 100, 100, 400, 401, 700, 900, 1000, 1024], dtype=torch.int32, device=dev)
    out = gm.grouped_mm(x, w, offs)  # lazy library setup outside the capture
    torch.cuda.synchronize()
    offs2 = torch.tensor([0, 0, 512, 512, 513, 600, 600, 1000, 1024], dtype=torch.int32, device=dev)
    s = torch.cuda.Stream()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        gm.grouped_mm(x, w, offs2, out=out)  # warm the stream
        torch.cuda.synchronize()
        with torch.cuda.graph(graph, stream=s):
            gm.grouped_mm(x, w, offs2, out=out)
    out.zero_()
    graph.replay()
    torch.cuda.synchronize()
    o = offs2.tolist()
    for e in range(G):
        if o[e + 1] > o[e]:
            ref = x[o[e]:o[e + 1]].float() @ w[e].float().t()
            assert _rel(out[o[e]:o[e + 1]], ref) < 1e-2, e
