"""ZeRO-Offload parity path (reference ``offload_optimizer`` cpu / nvme): host AdamW == device AdamW."""
import pytest
import torch

from distributed_llm_training_gpu_manager_amd import _host
from distributed_llm_training_gpu_manager_amd.models import get_config
from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine

pytestmark = pytest.mark.skipif(_host.lib() is None, reason="host runtime not built")


def _run(device, offload, tmp_path=None, stage=3, steps=3, clip=1.0):
    mc = get_config("llama-tiny")
    ec = EngineConfig(zero_stage=stage, micro_batch_size=2, seq_len=32, grad_accum=2, lr=3e-3, scheduler="constant",
                      init_device="cpu", grad_clip=clip, offload_optimizer=offload,
                      nvme_path=str(tmp_path) if tmp_path is not None else None)
    eng = ZeroEngine(mc, ec, torch.device(device))
    g = torch.Generator().manual_seed(7)
    losses = []
    for _ in range(steps):
        mbs = []
        for _ in range(2):
            t = torch.randint(0, mc.vocab_size, (2, 33), generator=g).to(device)
            mbs.append((t[:, :-1], t[:, 1:]))
        losses.append(float(eng.train_step(mbs)["loss"]))
    params = {k: v.float().cpu() for k, v in eng.full_params().items()}
    if eng.offload is not None:
        eng.offload.close()
    return losses, params, eng


@pytest.mark.parametrize("offload", ["cpu", "nvme"])
@pytest.mark.parametrize("clip", [0.0, 0.05])
def test_offload_matches_device_optimizer_cpu(tmp_path, offload, clip):
    ref_l, ref_p, _ = _run("cpu", "none", clip=clip)
    got_l, got_p, eng = _run("cpu", offload, tmp_path, clip=clip)
    assert eng.memory_report()["optimizer_state_host_GiB"] > 0
    # same math; fp32 rounding (FMA order) occasionally flips a bf16 compute-copy rounding, which Adam
    # then turns into at most a +-lr step on near-zero gradient elements
    assert ref_l[0] == got_l[0]
    for a, b in zip(ref_l, got_l):
        assert abs(a - b) < 1e-3 * max(1.0, abs(a)), (ref_l, got_l)
    for k, v in ref_p.items():
        d = (got_p[k] - v).abs()
        assert float(d.max()) <= 2 * 3e-3 * 3, k
        assert float((d > 3e-4).float().mean()) < 0.02, k


def test_offload_nan_step_is_skipped():
    mc = get_config("llama-tiny")
    ec = EngineConfig(zero_stage=1, micro_batch_size=1, seq_len=16, grad_accum=1, lr=1e-2, scheduler="constant",
                      init_device="cpu", offload_optimizer="cpu")
    eng = ZeroEngine(mc, ec, torch.device("cpu"))
    before = eng.master.clone()
    eng.fault_inject_nan = True
    t = torch.randint(0, mc.vocab_size, (1, 17))
    m = eng.train_step([(t[:, :-1], t[:, 1:])])
    assert float(m["nonfinite"]) > 0
    assert torch.equal(eng.master, before)


@pytest.mark.gpu
@pytest.mark.parametrize("offload", ["cpu", "nvme"])
def test_offload_matches_device_optimizer_gpu(tmp_path, offload):
    ref_l, ref_p, _ = _run("cuda", "none")
    got_l, got_p, _ = _run("cuda", offload, tmp_path)
    for a, b in zip(ref_l, got_l):
        assert abs(a - b) < 2e-3 * max(1.0, abs(a)), (ref_l, got_l)
    for k, v in ref_p.items():
        d = (got_p[k] - v).abs()
        assert float(d.max()) <= 2 * 3e-3 * 3, k
        assert float((d > 3e-4).float().mean()) < 0.02, k


def _grads(device, ckpt, cpu_ckpt):
    mc = get_config("llama-tiny")
    ec = EngineConfig(zero_stage=3, micro_batch_size=2, seq_len=32, grad_accum=2, lr=1e-3, scheduler="constant",
                      init_device="cpu", activation_checkpointing=ckpt, cpu_checkpointing=cpu_ckpt)
    eng = ZeroEngine(mc, ec, torch.device(device))
    g = torch.Generator().manual_seed(3)
    for i in range(2):
        t = torch.randint(0, mc.vocab_size, (2, 33), generator=g).to(device)
        eng.micro_step(t[:, :-1], t[:, 1:], first=i == 0, last=i == 1)
    return eng.grad_shard.float().cpu().clone()


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_activation_checkpointing_with_cpu_offload_is_exact(device):
    """Recompute (and recompute from host-offloaded inputs) reproduces the stored-activation gradients."""
    ref = _grads(device, False, False)
    assert torch.equal(_grads(device, True, False), ref)
    assert torch.equal(_grads(device, True, True), ref)


@pytest.mark.parametrize("nbuf", [3, 4, 6])
def test_nvme_swap_ring_matches_host_state(tmp_path, nbuf):
    """The AIO-swapped NVMe step (many chunks through a `buffer_count` ring) == the in-RAM host step,
    bitwise; the mapped views see the swapped state after each step."""
    from distributed_llm_training_gpu_manager_amd.parallel.offload import HostOffloadOptimizer
    n, chunk = 10_000 + 37, 1024  # 10 chunks, ragged tail
    dev = torch.device("cpu")
    ref = HostOffloadOptimizer(n, dev, "cpu", chunk_elems=chunk)
    nv = HostOffloadOptimizer(n, dev, "nvme", str(tmp_path), chunk_elems=chunk, buffer_count=nbuf, aio_threads=3,
                              aio_block_size=4096)
    init = torch.randn(n, generator=torch.Generator().manual_seed(0))
    for o in (ref, nv):
        o.master.copy_(init)
    p_ref, p_nv = torch.empty(n, dtype=torch.bfloat16), torch.empty(n, dtype=torch.bfloat16)
    g = torch.Generator().manual_seed(1)
    for step in range(1, 4):
        grad = torch.randn(n, generator=g)
        kw = dict(lr=1e-2, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.1, step=step, gscale=0.5)
        ref.step(grad, p_ref, **kw)
        nv.step(grad, p_nv, **kw)
        for a, b in ((ref.master, nv.master), (ref.exp_avg, nv.exp_avg), (ref.exp_avg_sq, nv.exp_avg_sq)):
            assert torch.equal(a, b)
        assert torch.equal(p_ref, p_nv)
    assert nv.swap_stats["read_GiB"] > 0 and nv.swap_stats["write_GiB"] > 0
    nv.close()


def test_aio_engine_roundtrip(tmp_path):
    """C++ AIO engine: overlapping async writes / reads, O_DIRECT when the filesystem allows it with a
    buffered fallback for unaligned pieces, reads past EOF return zeros."""
    aio = _host.Aio(4, 4096)
    for direct in (False, True):
        h = aio.open(str(tmp_path / f"f{int(direct)}"), 1 << 20, direct=direct)
        xs = [_host.aligned_empty(8192 + (777 if k == 3 else 0)) for k in range(4)]
        tks = []
        for k, x in enumerate(xs):
            x.copy_(torch.randn(x.numel(), generator=torch.Generator().manual_seed(k)))
            tks.append(aio.write(h, x, k * 65536))
        for tk in tks:
            aio.wait(tk)
        ys = [torch.zeros_like(x) for x in xs]  # not page-aligned: buffered fallback
        tks = [aio.read(h, y, k * 65536) for k, y in enumerate(ys)]
        for tk in tks:
            aio.wait(tk)
        for x, y in zip(xs, ys):
            assert torch.equal(x, y)
        tail = torch.full((4096,), 7.0)
        aio.wait(aio.read(h, tail, (1 << 20) + (1 << 22)))
        assert float(tail.abs().sum()) == 0.0
        aio.close(h, fsync=True)
    aio.shutdown()


def test_nvme_param_store_read_ahead(tmp_path):
    """offload_param=nvme read-ahead: the second pass over the same gather order is served by reads
    issued one access ahead; a write of the partition invalidates read-aheads in flight (new bytes are read)."""
    from distributed_llm_training_gpu_manager_amd.parallel.offload import NvmeParamStore
    n, piece = 4096, 512
    st = NvmeParamStore(n, torch.float32, str(tmp_path), 0, piece, buffer_count=4, aio_threads=2,
                        aio_block_size=4096)
    order = [(off, piece) for off in (0, 1024, 2048, 512, 3584)]

    def fill(base):
        st.write(lambda off, ln, slot: slot.copy_(torch.arange(off, off + ln, dtype=torch.float32) + base))

    for step, base in enumerate((0.0, 0.5, 7.0)):
        fill(base)
        for off, ln in order:
            i, t = st.read(off, ln)
            assert torch.equal(t, torch.arange(off, off + ln, dtype=torch.float32) + base), (step, off)
    # step 0 learns the order; steps 1 and 2 hit on every access after the first
    assert st.stats["read_ahead_hits"] == 2 * (len(order) - 1), st.stats
    st.close()


def test_touch_pages_maps_a_shared_file_and_sums_one_byte_per_page(tmp_path):
    """_host.touch_pages (csrc/host/ckpt_io.cpp): one byte read per 4 KiB page on several threads."""
    n = 40 << 20
    path = tmp_path / "snap"
    with open(path, "wb") as f:
        f.truncate(n)
    t = torch.from_file(str(path), shared=True, size=n, dtype=torch.uint8)
    t[0], t[4096 * 7], t[4096 * 7 + 1], t[n - 4096] = 3, 5, 100, 11  # the +1 byte is not on a page start
    assert _host.touch_pages(t, 4) == 3 + 5 + 11
    assert _host.touch_pages(t[:8192], 16) == 3


def test_populate_pages_maps_a_reserved_shm_file_writable_and_keeps_its_bytes(tmp_path):
    """_host.populate_pages (MADV_POPULATE_WRITE on threads, csrc/host/ckpt_io.cpp): the snapshot pipeline's map
    stage. It must not change any byte (a restore source may already be in the file) and must cover every slice,
    the last partial one included."""
    import os
    n = (130 << 20) + 4096 * 3  # three 64 MiB slices, the last one short
    path = "/dev/shm/dlgm-test-populate.snap" if os.path.isdir("/dev/shm") else str(tmp_path / "snap")
    fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o600)
    try:
        os.ftruncate(fd, n)
        os.posix_fallocate(fd, 0, n)
        os.close(fd)
        t = torch.from_file(path, shared=True, size=n, dtype=torch.uint8)
        t[0], t[(64 << 20) + 5], t[n - 1] = 7, 9, 11
        ok = _host.populate_pages(t, 8)
        assert ok or _host.lib() is None  # Linux >= 5.14 with the host library built
        assert (int(t[0]), int(t[(64 << 20) + 5]), int(t[n - 1])) == (7, 9, 11)
        assert int(t.sum()) == 7 + 9 + 11
        del t
    finally:
        if os.path.exists(path):
            os.unlink(path)
