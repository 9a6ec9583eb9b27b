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
