"""CPU contract of moe_permute (the device kernel is checked against this in test_kernels_gpu.py)."""
import torch

from distributed_llm_training_gpu_manager_amd.ops.moe import moe_permute


def test_moe_permute_contract():
    torch.manual_seed(0)
    T, K, E = 257, 2, 8
    topi = torch.randint(0, E, (T, K))
    topi[topi == 5] = 1
    off, pos, src = moe_permute(topi, E)
    assert off[0] == 0 and off[-1] == T * K and off[6] == off[5]
    flat = topi.reshape(-1)
    # sorted row r holds the slot whose expert owns the range containing r, tokens in order
    for e in range(E):
        rows = torch.arange(int(off[e]), int(off[e + 1]))
        slots = torch.nonzero(flat == e).flatten()
        assert torch.equal(pos.reshape(-1)[slots], rows)
        assert torch.equal(src[rows], slots // K)


def test_ep_regroup_index_on_device_matches_host_construction():
    """The EP dispatcher's [source rank][local expert] -> [local expert][source rank] permutation is built on
    the device from the count matrix (no host list, no index copy): it equals the block-by-block host build."""
    import torch
    from distributed_llm_training_gpu_manager_amd.parallel.ep import _regroup_index

    g = torch.Generator().manual_seed(0)
    for W, El in ((2, 4), (4, 2), (8, 1), (3, 5)):
        mat = torch.randint(0, 6, (W, El), generator=g)
        mat[0, 0] = 0  # an empty block
        flat = mat.reshape(-1)
        starts = (torch.cumsum(flat, 0) - flat).view(W, El)
        idx = [torch.arange(int(starts[s, e]), int(starts[s, e] + mat[s, e])) for e in range(El) for s in range(W)]
        want = torch.cat(idx) if idx else torch.zeros(0, dtype=torch.long)
        got = _regroup_index(mat.to(torch.int32), int(mat.sum()))
        assert torch.equal(got, want), (W, El)
