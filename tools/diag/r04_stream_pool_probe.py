"""Does the Mixtral EP-4 async-shadow result depend on which pool streams the communicators get? Advance
PyTorch's stream pool by k before each run (k = 0..31) and group the results by bit-equality."""
import sys

import torch

sys.path.insert(0, ".")
from tests.test_shadow_async_gpu import _run  # noqa: E402

KW = dict(zero_stage=3, expert_parallel_size=4, local_grad_accum=False)
sync, _ = _run("mixtral-tiny", 4, False, optimizer_overlap=False, **KW)
classes = []
for k in range(32):
    for _ in range(k):
        torch.cuda.Stream()
    for ov in (False, True):
        got, _ = _run("mixtral-tiny", 4, True, optimizer_overlap=ov, **KW)
        hit = next((ci for ci, (rep, _) in enumerate(classes) if all(torch.equal(rep[x], got[x]) for x in got)), None)
        if hit is None:
            classes.append((got, []))
            hit = len(classes) - 1
        classes[hit][1].append((k, ov))
        print(k, ov, "class", hit, flush=True)
for ci, (rep, ks) in enumerate(classes):
    print("class", ci, "== sync:", all(torch.equal(rep[x], sync[x]) for x in rep), "members:", ks)
