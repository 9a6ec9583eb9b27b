"""Does any engine path read memory it never wrote? Run the Mixtral EP-4 / Llama cases on a clean caching
allocator, then again after filling the allocator's cached blocks with a poison value: results must not change."""
import sys

import torch

sys.path.insert(0, ".")
from tests.test_shadow_async_gpu import _run  # noqa: E402


def poison(val):
    torch.cuda.synchronize()
    keep = []
    for mb in (1, 2, 4, 8, 16, 32, 64, 128, 256, 512):
        for _ in range(6):
            keep.append(torch.full((mb << 18,), val, device="cuda"))
    for sz in (512, 4096, 65536, 1 << 20):
        for _ in range(32):
            keep.append(torch.full((sz // 4,), val, device="cuda"))
    torch.cuda.synchronize()
    del keep  # blocks stay cached by the allocator, holding the poison


CASES = [
    ("mixtral-tiny", 4, dict(zero_stage=3, expert_parallel_size=4, local_grad_accum=False)),
    ("mixtral-tiny", 4, dict(zero_stage=2, expert_parallel_size=4, local_grad_accum=False)),
    ("llama-tiny", 4, dict(zero_stage=3, local_grad_accum=False)),
]
for model, world, kw in CASES:
    for ov in (False, True):
        torch.cuda.empty_cache()
        clean, _ = _run(model, world, True, optimizer_overlap=ov, **kw)
        for val in (float("nan"), 1e4):
            torch.cuda.empty_cache()
            poison(val)
            got, _ = _run(model, world, True, optimizer_overlap=ov, **kw)
            diff = {k: float((clean[k].float() - got[k].float()).abs().max()) for k in clean
                    if not torch.equal(clean[k], got[k])}
            print(model, kw, "overlap", ov, "poison", val, "identical" if not diff else diff, flush=True)
