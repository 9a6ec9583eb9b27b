"""utils/streams.owned_stream leasing (round-robin slots isolated owners only while <= 16 of
a kind were live): a live owner's stream is never handed to another owner; a dead owner's stream is reused."""
import gc

import torch

from distributed_llm_training_gpu_manager_amd.utils import streams as S


class _FakeStream:
    n = 0

    def __init__(self):
        _FakeStream.n += 1
        self.cuda_stream = 0x5000 + _FakeStream.n


class _Owner:
    pass


def test_live_owners_never_share_and_dead_ones_give_back(monkeypatch):
    monkeypatch.setattr(S, "_new_stream", lambda idx: _FakeStream())
    monkeypatch.setattr(S, "_POOL", False)
    dev = torch.device("cuda", 0)
    kind = "lease-test"
    owners = [_Owner() for _ in range(40)]  # more than the 16 round-robin slots
    got = [S.owned_stream(dev, kind, owner=o) for o in owners]
    assert len({id(s) for s in got}) == 40
    dead = got[7]
    del owners[7]
    gc.collect()
    keep = _Owner()
    again = S.owned_stream(dev, kind, owner=keep)
    assert again is dead  # the dead owner's stream, not a 41st one
    other = S.owned_stream(dev, "lease-test-other", owner=_Owner())
    assert other is not dead  # free lists are per kind
    del keep
