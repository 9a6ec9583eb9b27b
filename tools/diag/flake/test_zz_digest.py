"""Round-5 flake probe: after the GPU selection that precedes the Mixtral EP-4
overlapped-optimizer mismatch, run the non-overlapped reference engine twice (one step, GA 2) under a
TorchDispatchMode that synchronises after every aten / dlgm op and digests each tensor it touched, then report
the first op whose digests differ between the first and the second engine.

Copied into tests/ by the gpurun command (never collected from tools/)."""
import hashlib
import json
import os

import pytest
import torch
from torch.utils._python_dispatch import TorchDispatchMode
from torch.utils._pytree import tree_leaves

from distributed_llm_training_gpu_manager_amd.models import get_config
from distributed_llm_training_gpu_manager_amd.parallel.comm import ShadowComm
from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine

pytestmark = pytest.mark.gpu
SKIP = ("empty", "empty_like", "empty_strided", "new_empty", "new_empty_strided", "_local_scalar_dense")
OUT = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "digest")


def _dig(t):
    b = t.detach().contiguous().view(-1)
    b = b.view(torch.uint8) if b.dtype != torch.bool else b.to(torch.uint8)
    return hashlib.sha1(b.cpu().numpy().tobytes()).hexdigest()[:16]


class Digest(TorchDispatchMode):
    def __init__(self, keep=4000):
        super().__init__()
        self.log, self.data, self.keep = [], [], keep

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = func.__name__ if hasattr(func, "__name__") else str(func)
        if any(name.startswith(s) for s in SKIP):
            return out
        torch.cuda.synchronize()
        ts = [t for t in tree_leaves((out, args, kwargs or {})) if isinstance(t, torch.Tensor) and t.is_cuda]
        self.log.append((str(func), [(tuple(t.shape), str(t.dtype), _dig(t)) for t in ts]))
        if len(self.data) < self.keep:
            self.data.append([t.detach().float().cpu().clone() if t.numel() < (1 << 22) and t.is_floating_point()
                              else None for t in ts])
        return out


def _engine_run(mode, steps=3):
    dev = torch.device("cuda", 0)
    mc = get_config("mixtral-tiny")
    ec = EngineConfig(micro_batch_size=2, seq_len=64, grad_accum=2, lr=1e-3, scheduler="constant", grad_clip=1.0,
                      zero_stage=3, expert_parallel_size=4, local_grad_accum=False, optimizer_overlap=False)
    comm = ShadowComm(4, 0, async_mode=True, delay_cycles=200_000)
    eng = ZeroEngine(mc, ec, dev, comm)
    g = torch.Generator().manual_seed(3)
    with mode:
        for _ in range(steps):
            mbs = []
            for _ in range(2):
                t = torch.randint(0, mc.vocab_size, (2, 65), generator=g).to(dev)
                mbs.append((t[:, :-1].contiguous(), t[:, 1:].contiguous()))
            eng.train_step(mbs)
        torch.cuda.synchronize()
    return {k: getattr(eng, k).detach().cpu().clone() for k in ("master", "grad_shard")}


def test_zz_digest():
    os.makedirs(OUT, exist_ok=True)
    runs = []
    import contextlib
    plain = os.environ.get("DIGEST", "1") == "0"
    for i in range(3):
        m = Digest()
        st = _engine_run(contextlib.nullcontext() if plain else m)
        runs.append((m, st))
    rep = {"n_ops": [len(m.log) for m, _ in runs],
           "state_equal": {f"{a}{b}": all(torch.equal(runs[a][1][k], runs[b][1][k]) for k in runs[a][1])
                           for a, b in ((0, 1), (1, 2), (0, 2))}}
    first = []
    A, B = runs[0][0], runs[1][0]
    for i, (la, lb) in enumerate(zip(A.log, B.log)):
        if la != lb:
            ent = {"i": i, "op": la[0], "opB": lb[0], "a": la[1], "b": lb[1]}
            if i < len(A.data) and i < len(B.data):
                diffs = []
                for ta, tb in zip(A.data[i], B.data[i]):
                    if ta is None or tb is None or ta.shape != tb.shape:
                        diffs.append(None)
                        continue
                    d = (ta - tb).abs()
                    nz = (d > 0) | (ta.isnan() != tb.isnan())
                    rows = nz.reshape(nz.shape[0], -1).any(1).nonzero().flatten()[:16].tolist() if nz.dim() else []
                    diffs.append({"n": int(nz.sum()), "max": float(torch.nan_to_num(d, nan=-1.0).max()),
                                  "rows": rows, "nan_a": int(ta.isnan().sum()), "nan_b": int(tb.isnan().sum())})
                ent["diff"] = diffs
            first.append(ent)
            if len(first) >= 12:
                break
    rep["first_diffs"] = first
    rep["ops_context"] = [A.log[j][0] for j in range(max(0, (first[0]["i"] if first else 0) - 15),
                                                    (first[0]["i"] + 3) if first else 0)]
    with open(os.path.join(OUT, f"digest_report_{os.environ.get('DIGEST', '1')}.json"), "w") as f:
        json.dump(rep, f, indent=1)
    print(json.dumps({k: rep[k] for k in ("n_ops", "state_equal")}))
    print(json.dumps(first[:3])[:4000])
