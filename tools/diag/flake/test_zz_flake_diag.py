"""Run after the GPU selection that precedes the Mixtral EP-4 overlapped-optimizer mismatch: which of ref / got is
unstable, and in which groups and state tensors."""
import pytest
import torch

from tests.test_shadow_async_gpu import _run

pytestmark = pytest.mark.gpu
KW = dict(zero_stage=3, expert_parallel_size=4, local_grad_accum=False)
GROUPS = [(0, 0, 32768), (1, 32768, 49536), (2, 82304, 196608), (3, 278912, 49536), (4, 328448, 196608),
          (5, 525056, 32832)]


def _cmp(a, b):
    out = {}
    for k in a:
        d = (a[k].float() - b[k].float()).abs()
        if d.max() > 0:
            out[k] = [(gi, float(d[o:o + n].max()), int((d[o:o + n] > 0).sum())) for gi, o, n in GROUPS
                      if d[o:o + n].max() > 0]
    return out or "identical"


def test_zz_flake_diag():
    r1, _ = _run("mixtral-tiny", 4, True, optimizer_overlap=False, **KW)
    g1, _ = _run("mixtral-tiny", 4, True, opt_delay=2_000_000, optimizer_overlap=True, **KW)
    r2, _ = _run("mixtral-tiny", 4, True, optimizer_overlap=False, **KW)
    g2, _ = _run("mixtral-tiny", 4, True, opt_delay=0, optimizer_overlap=True, **KW)
    s1, _ = _run("mixtral-tiny", 4, False, optimizer_overlap=False, **KW)
    print("\nr1 vs g1", _cmp(r1, g1))
    print("r1 vs r2", _cmp(r1, r2))
    print("r1 vs g2", _cmp(r1, g2))
    print("r1 vs sync", _cmp(r1, s1))
    print("g1 vs sync", _cmp(g1, s1))
