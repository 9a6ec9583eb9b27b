"""Round 5: how fast can a /dev/shm snapshot file be made resident on the GPU box, and what does a new process's
first big device allocation cost after another process freed that memory (the 4.6-4.9 s engine construction of
every process but the first in a call)?
  host: posix_fallocate (1 thread), MADV_POPULATE_WRITE on 16 disjoint ranges of the mapping (16 threads), the
        same after MADV_HUGEPAGE, 16-thread first-touch writes; the THP settings of the box
  device: 96 GiB allocated clean, freed back to the driver (empty_cache), allocated again"""
import ctypes
import json
import mmap
import os
import threading
import time

import torch

G = 1 << 30
SIZE = int(float(os.environ.get("SIZE", "32")) * G)
NT = 16
libc = ctypes.CDLL("libc.so.6", use_errno=True)
libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
MADV_HUGEPAGE, MADV_POPULATE_WRITE = 14, 23
res = {"GiB": SIZE / G}
for k in ("enabled", "shmem_enabled", "defrag"):
    try:
        res["thp_" + k] = open(f"/sys/kernel/mm/transparent_hugepage/{k}").read().strip()
    except OSError as e:
        res["thp_" + k] = str(e)


def mapped(path):
    fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o600)
    os.ftruncate(fd, SIZE)
    m = mmap.mmap(fd, SIZE, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
    os.close(fd)
    buf = ctypes.c_char.from_buffer(m)
    return m, buf, ctypes.addressof(buf)


def threads(fn):
    step = SIZE // NT
    ths = [threading.Thread(target=fn, args=(i * step, step)) for i in range(NT)]
    t0 = time.time()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return round(time.time() - t0, 2)


def case(name, huge=False, how="populate"):
    path = f"/dev/shm/dlgm-prefault-{name}"
    m, buf, addr = mapped(path)
    try:
        if huge:
            res[name + "_madv_huge_rc"] = libc.madvise(addr, SIZE, MADV_HUGEPAGE)
        if how == "populate":
            rcs = []
            dt = threads(lambda off, ln: rcs.append(libc.madvise(addr + off, ln, MADV_POPULATE_WRITE)))
            res[name + "_rc"] = sorted(set(rcs))
        elif how == "touch":
            def touch(off, ln):
                ctypes.memset(addr + off, 0, ln)
            dt = threads(touch)
        else:
            fd = os.open(path, os.O_RDWR)
            t0 = time.time()
            os.posix_fallocate(fd, 0, SIZE)
            dt = round(time.time() - t0, 2)
            os.close(fd)
        res[name + "_s"] = dt
        res[name + "_GBps"] = round(SIZE / dt / 1e9, 1) if dt > 0 else None
        try:
            smaps = open(f"/proc/{os.getpid()}/smaps_rollup").read()
            res[name + "_shmem_pmd_kB"] = [ln for ln in smaps.splitlines() if "ShmemPmdMapped" in ln]
        except OSError:
            pass
    finally:
        del buf
        m.close()
        os.unlink(path)


case("fallocate_1t", how="fallocate")
case("populate_16t")
case("populate_huge_16t", huge=True)
case("touch_16t", how="touch")
print(json.dumps(res), flush=True)

dev = torch.device("cuda", 0)
if not torch.cuda.is_available():
    raise SystemExit(0)
torch.cuda.init()
n = int(float(os.environ.get("VRAM", "96")) * G)
for name in ("vram_first", "vram_again"):
    torch.cuda.synchronize()
    t0 = time.time()
    bufs = [torch.empty(G, dtype=torch.uint8, device=dev) for _ in range(n // G)]
    torch.cuda.synchronize()
    res[name + "_alloc_s"] = round(time.time() - t0, 2)
    t0 = time.time()
    for b in bufs:
        b.fill_(1)
    torch.cuda.synchronize()
    res[name + "_fill_s"] = round(time.time() - t0, 2)
    del bufs
    torch.cuda.empty_cache()
print(json.dumps(res), flush=True)
os.makedirs("gpurun_out/digest", exist_ok=True)
with open("gpurun_out/digest/prefault_bench.json", "w") as f:
    json.dump(res, f, indent=1)
