"""Repeat the Mixtral EP-4 overlapped-optimizer bit-identity case and name the parameter groups that differ."""
import sys

import torch

sys.path.insert(0, ".")
from tests.test_shadow_async_gpu import _run  # noqa: E402
from distributed_llm_training_gpu_manager_amd.models import get_config  # noqa: E402
from distributed_llm_training_gpu_manager_amd.parallel.comm import ShadowComm  # noqa: E402
from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine  # noqa: E402

kw = dict(zero_stage=3, expert_parallel_size=4, local_grad_accum=False)
mc = get_config("mixtral-tiny")
ec = EngineConfig(micro_batch_size=2, seq_len=64, grad_accum=2)
for k, v in kw.items():
    setattr(ec, k, v)
eng = ZeroEngine(mc, ec, torch.device("cuda", 0), ShadowComm(4, 0, async_mode=True))
groups = [(g.idx, g.kind, g.P, g.shard_off, g.shard_numel, [s.name for s in g.specs][:3]) for g in eng.groups]
print("groups", groups, "order", eng._opt_order, flush=True)
del eng
ref, _ = _run("mixtral-tiny", 4, True, optimizer_overlap=False, **kw)
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    for od in (2_000_000, 20_000_000, 100_000_000):
        got, _ = _run("mixtral-tiny", 4, True, opt_delay=od, optimizer_overlap=True, **kw)
        bad = {}
        for k in ref:
            d = (ref[k].float() - got[k].float()).abs()
            if d.max() > 0:
                bad[k] = [(gi, kind, float(d[off:off + n].max())) for gi, kind, P, off, n, _ in groups
                          if n and d[off:off + n].max() > 0]
        print("rep", rep, "opt_delay", od, "identical" if not bad else bad, flush=True)
    ref2, _ = _run("mixtral-tiny", 4, True, optimizer_overlap=False, **kw)
    print("rep", rep, "ref vs ref", all(torch.equal(ref[k], ref2[k]) for k in ref), flush=True)
