"""Shadow xGMI-mesh heap pool (parallel/xgmi_mesh.py): best fit by size, removal by identity (tensors are never
compared with ==), one pool per (device, memory kind). The GPU side is tests/test_xgmi_mesh_gpu.py."""
import torch

from distributed_llm_training_gpu_manager_amd.parallel import xgmi_mesh as X


def test_pool_takes_the_smallest_heap_that_fits_and_keeps_the_rest():
    key = (97, 1)  # a device index nothing else uses
    X._HEAP_POOL.pop(key, None)
    a, b, c = torch.zeros(10, dtype=torch.uint8), torch.zeros(30, dtype=torch.uint8), torch.zeros(20, dtype=torch.uint8)
    for t in (a, b, c):
        X._pool_give(*key, t)
    assert X._pool_take(*key, 15) is c
    assert X._pool_take(*key, 15) is b
    assert X._pool_take(*key, 15) is None
    assert X._pool_take(*key, 10) is a
    assert X._pool_take(97, 0, 1) is None  # another memory kind: its own pool
    X._HEAP_POOL.pop(key, None)
