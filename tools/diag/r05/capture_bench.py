"""Round 5: end-to-end capture of SIZE GiB of device memory into a FRESH /dev/shm file (what an early spot notice
costs), by strategy. The drill's pipeline ran at ~5.5 GB/s, bounded by the page-mapping stage (a reserved tmpfs
page is zeroed at its first touch; one thread ~5.4 GB/s on this host, populate_bench.py).
  pipeT    reserve thread (posix_fallocate, 1 GiB pieces) | map stage (_host.touch_pages on T threads) | caller:
           hipHostRegister of each mapped piece, then its D2H queued (the checkpointer's _lock_and_dma)
  pwrite   D2H into 4 pinned 256 MiB slots; each slot pwrite()n into the unmapped file by the host runtime's
           threads (a full-page write into a tmpfs file needs no zeroing)
  pwritef  the same with a reserve thread running ahead (posix_fallocate)
Every strategy's file is checked against the device bytes (CRC32C of the whole file vs of a D2H copy)."""
import ctypes
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.getcwd())
from distributed_llm_training_gpu_manager_amd import _host  # noqa: E402

G = 1 << 30
SIZE = int(float(os.environ.get("SIZE", "24")) * G)
SLOT = 256 << 20
PW_CHUNK = 16 << 20
hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
dev = torch.device("cuda", 0)
src = torch.randint(0, 256, (SIZE,), dtype=torch.uint8, device=dev)
stream = torch.cuda.Stream(dev)
want = None
res = {"GiB": SIZE / G, "threads": _host.THREADS}


def gbps(dt):
    return round(SIZE / dt / 1e9, 1)


def check(name, path):
    global want
    if want is None:
        host = torch.empty(SIZE, dtype=torch.uint8, pin_memory=True)
        host.copy_(src)
        want = _host.crc32c_chunks(host)
        del host
    got = _host.crc32c_chunks(torch.from_file(path, shared=False, size=SIZE, dtype=torch.uint8))
    res[name + "_ok"] = got == want


def pipe(name, nthreads):
    path = f"/dev/shm/dlgm-capbench-{name}"
    fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o600)
    os.ftruncate(fd, SIZE)
    snap = torch.from_file(path, shared=True, size=SIZE, dtype=torch.uint8)
    st = {"falloc": 0, "mapped": 0}
    t0 = time.time()

    def reserve():
        for off in range(0, SIZE, G):
            os.posix_fallocate(fd, off, G)
            st["falloc"] = off + G

    def mapper():
        for off in range(0, SIZE, G):
            while st["falloc"] < off + G:
                time.sleep(0.0005)
            _host.touch_pages(snap[off:off + G], nthreads)
            st["mapped"] = off + G
    ths = [threading.Thread(target=reserve), threading.Thread(target=mapper)]
    for t in ths:
        t.start()
    regs = []
    for off in range(0, SIZE, G):
        while st["mapped"] < off + G:
            time.sleep(0.0005)
        assert hip.hipHostRegister(snap.data_ptr() + off, G, 0) == 0
        regs.append(snap.data_ptr() + off)
        with torch.cuda.stream(stream):
            snap[off:off + G].copy_(src[off:off + G], non_blocking=True)
    stream.synchronize()
    res[name + "_GBps"] = gbps(time.time() - t0)
    for t in ths:
        t.join()
    for r in regs:
        hip.hipHostUnregister(r)
    os.close(fd)
    del snap
    check(name, path)
    os.unlink(path)


def pwrite(name, ahead):
    L = _host.lib()
    path = f"/dev/shm/dlgm-capbench-{name}"
    fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o600)
    os.ftruncate(fd, SIZE)
    slots = [torch.empty(SLOT, dtype=torch.uint8, pin_memory=True) for _ in range(4)]
    st = {"falloc": SIZE if not ahead else 0}
    t0 = time.time()
    th = None
    if ahead:
        def reserve():
            for off in range(0, SIZE, G):
                os.posix_fallocate(fd, off, G)
                st["falloc"] = off + G
        th = threading.Thread(target=reserve)
        th.start()
    pend = []

    def drain():
        k, off, ev = pend.pop(0)
        ev.synchronize()
        rc = L.dlgm_pwrite_at(fd, ctypes.c_void_p(slots[k % 4].data_ptr()), SLOT, off, PW_CHUNK, _host.THREADS, None)
        assert rc == 0, rc
    for k, off in enumerate(range(0, SIZE, SLOT)):
        if len(pend) == 4:
            drain()
        with torch.cuda.stream(stream):
            slots[k % 4].copy_(src[off:off + SLOT], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
        pend.append((k, off, ev))
    while pend:
        drain()
    res[name + "_GBps"] = gbps(time.time() - t0)
    if th is not None:
        th.join()
    os.close(fd)
    check(name, path)
    os.unlink(path)


for c in os.environ.get("CASES", "pipe1,pipe8,pipe16,pwrite,pwritef").split(","):
    if c.startswith("pipe"):
        pipe(c, int(c[4:]))
    else:
        pwrite(c, c.endswith("f"))
    print(c, {k: v for k, v in res.items() if k.startswith(c + "_")}, flush=True)
os.makedirs("gpurun_out/digest", exist_ok=True)
with open("gpurun_out/digest/capture_bench.json", "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps(res))
