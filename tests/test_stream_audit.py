"""The stream-ordering audit's clock model (utils/stream_audit.py HazardModel) on synthetic stream histories (CPU),
and on the GPU: real side-stream bugs it must name, the engine's own streams it must pass."""
import pytest
import torch

from distributed_llm_training_gpu_manager_amd.utils.stream_audit import HazardModel, stream_audit

C, S = "compute", "side"


class Box:
    alive = True


def _rec(m, key, base, n, stream, box):
    return m.storage(key, base, n, stream, lambda: box.alive)


def _acc(m, rec, s, write, lo=0, hi=None, what="op"):
    t = m.enqueue(s)
    m.access(rec, lo, rec.nbytes if hi is None else hi, s, t, write, what)


def test_raw_without_wait_is_reported_and_an_event_wait_clears_it():
    m = HazardModel()
    a = Box()
    r = _rec(m, 1, 0x1000, 256, C, a)
    _acc(m, r, S, True, what="side_write")
    _acc(m, r, C, False, what="compute_read")
    assert [h.kind for h in m.hazards] == ["RAW"]
    m2 = HazardModel()
    r = _rec(m2, 1, 0x1000, 256, C, a)
    _acc(m2, r, S, True)
    m2.wait(C, m2.snapshot(S))
    _acc(m2, r, C, False)
    assert not m2.hazards


def test_war_and_waw_and_disjoint_ranges():
    m = HazardModel()
    r = _rec(m, 1, 0x1000, 1024, C, Box())
    _acc(m, r, C, False, 0, 512)
    _acc(m, r, S, True, 512, 1024)  # disjoint bytes: no conflict
    assert not m.hazards
    _acc(m, r, S, True, 0, 256)  # overwrites bytes compute read without waiting for it
    assert [h.kind for h in m.hazards] == ["WAR"]
    _acc(m, r, C, True, 600, 700)  # writes bytes the side stream wrote, unordered
    assert [h.kind for h in m.hazards] == ["WAR", "WAW"]


def test_same_stream_and_host_sync_never_race():
    m = HazardModel()
    r = _rec(m, 1, 0x1000, 64, C, Box())
    _acc(m, r, S, True)
    _acc(m, r, S, False)
    m.device_sync()
    _acc(m, r, C, True)
    assert not m.hazards


def test_freed_block_reused_while_another_stream_still_reads_it():
    """The caching-allocator hazard: a tensor allocated on compute and read on a side stream is freed without
    record_stream; compute's next allocation gets the block and writes it while the side read may be pending."""
    m = HazardModel()
    old = Box()
    r = _rec(m, 1, 0x1000, 4096, C, old)
    _acc(m, r, C, True, what="producer")
    m.wait(S, m.snapshot(C))
    _acc(m, r, S, False, what="side_consumer")
    old.alive = False  # freed on the host
    r2 = _rec(m, 2, 0x1800, 1024, C, Box())  # a new tensor in part of the old block
    _acc(m, r2, C, True, what="next_writer")
    assert [h.kind for h in m.hazards] == ["reuse"]
    assert "side_consumer" not in m.hazards[0].second and "next_writer" in m.hazards[0].second


@pytest.mark.parametrize("fix", ["record_stream", "wait_consumer", "host_sync"])
def test_reuse_is_clean_with_each_legal_edge(fix):
    m = HazardModel()
    old = Box()
    r = _rec(m, 1, 0x1000, 4096, C, old)
    _acc(m, r, C, True)
    m.wait(S, m.snapshot(C))
    _acc(m, r, S, False)
    if fix == "record_stream":
        m.record_stream(r, S)
    elif fix == "wait_consumer":
        m.wait(C, m.snapshot(S))
    else:
        m.device_sync()
    old.alive = False
    r2 = _rec(m, 2, 0x1000, 4096, C, Box())
    _acc(m, r2, C, True)
    assert not m.hazards, m.report()


def test_recycled_storage_key_still_checks_reuse():
    m = HazardModel()
    old = Box()
    r = _rec(m, 7, 0x4000, 512, C, old)
    _acc(m, r, S, False, what="side_read")
    old.alive = False
    r2 = _rec(m, 7, 0x4000, 512, C, Box())  # same storage key and address, new tensor
    assert r2 is not r
    _acc(m, r2, C, True)
    assert [h.kind for h in m.hazards] == ["reuse"]


def test_new_storage_beside_a_dead_one_is_not_a_reuse():
    m = HazardModel()
    old = Box()
    r = _rec(m, 1, 0x1000, 256, C, old)
    _acc(m, r, S, False)
    old.alive = False
    r2 = _rec(m, 2, 0x1100, 256, C, Box())  # starts where the dead one ended
    _acc(m, r2, C, True)
    assert not m.hazards


def test_dispatch_binding_reads_schemas_and_skips_views():
    """The TorchDispatchMode layer on CPU tensors with a test stream key: outputs are writes, in-place arguments are
    writes, views touch nothing, and a missing wait between two streams is named with both ops."""
    from distributed_llm_training_gpu_manager_amd.utils.stream_audit import _make_mode
    m = HazardModel()
    cur = {"s": C}
    with _make_mode(m, fake_stream=lambda: cur["s"]):
        x = torch.randn(1 << 10)
        cur["s"] = S
        m.wait(S, m.snapshot(C))
        y = x * 2  # side stream writes y
        v = y[:16]  # a view: no access
        cur["s"] = C
        assert not m.hazards
        z = v + 1  # compute reads y's bytes without waiting for the side stream
        assert [h.kind for h in m.hazards] == ["RAW"] and "mul" in m.hazards[0].first
        m.wait(C, m.snapshot(S))
        x.add_(z.sum())  # in-place write on compute, ordered after the side read of x by the wait above
    assert len(m.hazards) == 1, m.report()


# ------------------------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.no_stream_audit
def test_audit_names_a_missing_wait_and_a_missing_record_stream_on_the_gpu():
    dev = torch.device("cuda", 0)
    side = torch.cuda.Stream(dev)
    with stream_audit() as a:
        x = torch.randn(1 << 16, device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            y = x * 2  # allocated on the side stream
        z = y + 1  # consumed on compute without waiting for the side stream
        del z
    assert any(h.kind == "RAW" for h in a.hazards), (a.report(), {r.name: r.accesses for r in a.recs.values()},
                                                    a.vc, a.host)
    del x, y
    torch.cuda.synchronize()
    n = (3 << 16) + 512  # a size nothing else in this process allocates: the next same-size block is x's
    with stream_audit() as b:
        x = torch.randn(n, device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            s = x.sum()
        ptr = x.data_ptr()
        del x  # no record_stream: compute may reuse the block while the side stream reads it
        w = torch.empty(n, device=dev)
        assert w.data_ptr() == ptr  # the caching allocator handed the block straight back
        w.fill_(1.0)
        torch.cuda.current_stream(dev).wait_stream(side)
        del s, w
    assert any(h.kind == "reuse" for h in b.hazards), b.report()
    torch.cuda.synchronize()
    n += 512
    with stream_audit() as c:
        x = torch.randn(n, device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            s = x.sum()
        x.record_stream(side)
        del x
        w = torch.empty(n, device=dev)
        w.fill_(1.0)
        torch.cuda.current_stream(dev).wait_stream(side)
        float(s)
    assert not c.hazards, c.report()


def test_host_key_ops_complete_on_return():
    """CPU ops on pinned memory (stream key HOST) are complete when they return: a later device copy on any stream is
    ordered after them; but a host write over bytes an earlier async copy still reads is a WAR race."""
    from distributed_llm_training_gpu_manager_amd.utils.stream_audit import HOST
    m = HazardModel()
    r = _rec(m, 1, 0x9000, 256, HOST, Box())
    t = m.enqueue(HOST)
    m.access(r, 0, 256, HOST, t, True, "host_fill")
    m.host_sync({HOST: t})
    _acc(m, r, S, False, what="h2d_read")  # queued after the host wrote: ordered
    assert not m.hazards
    t = m.enqueue(HOST)
    m.access(r, 0, 64, HOST, t, True, "host_overwrite")  # the H2D may not have run yet
    assert [h.kind for h in m.hazards] == ["WAR"] and "h2d_read" in m.hazards[0].first


@pytest.mark.gpu
@pytest.mark.no_stream_audit
def test_audit_tracks_pinned_host_buffers_on_the_gpu():
    """A D2H into a pinned buffer on one stream and an H2D out of it on another, without an event between them: the
    RAW on page-locked host memory is named; with the event it is clean."""
    dev = torch.device("cuda", 0)
    side = torch.cuda.Stream(dev)
    host = torch.empty(1 << 16, pin_memory=True)
    for ordered in (False, True):
        with stream_audit() as a:
            x = torch.randn(1 << 16, device=dev)
            host.copy_(x, non_blocking=True)  # D2H on compute
            ev = torch.cuda.Event()
            ev.record()
            with torch.cuda.stream(side):
                if ordered:
                    side.wait_event(ev)
                y = torch.empty(1 << 16, device=dev)
                y.copy_(host, non_blocking=True)  # H2D on the side stream
            torch.cuda.synchronize()
        kinds = [h.kind for h in a.hazards]
        assert kinds == ([] if ordered else ["RAW"]), a.report()
        assert ordered or "pinned" in a.hazards[0].storage
