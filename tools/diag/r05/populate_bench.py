"""Round 5: can a fresh /dev/shm snapshot file be made DMA-ready faster than posix_fallocate's ~5-19 GB/s?
posix_fallocate on tmpfs holds the inode lock for the whole call, so threads cannot split it; page faults on
disjoint ranges of one MAP_SHARED mapping can run in parallel. Cases (SIZE GiB each, then hipHostRegister in
1 GiB pieces, optionally with BUSY_GIB of device memory allocated and a GEMM loop running, as in the trainer):
  falloc1        posix_fallocate, one thread, then read-map one byte per page, then register (today's stages)
  fallocN        posix_fallocate of disjoint 1 GiB ranges from N threads
  popwN          MADV_POPULATE_WRITE of disjoint 1 GiB ranges from N threads (allocates, zeroes and maps)
  touchN         one byte written per 4 KiB page from N threads (numpy strided store)
  fregN          posix_fallocate from N threads, then register the reserved but unmapped pages
  hugeN          MADV_HUGEPAGE on the mapping, then MADV_POPULATE_WRITE from N threads"""
import ctypes
import json
import mmap
import os
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

G = 1 << 30
SIZE = int(float(os.environ.get("SIZE", "24")) * G)
BUSY = float(os.environ.get("BUSY_GIB", "0"))
libc = ctypes.CDLL("libc.so.6", use_errno=True)
libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
MADV_POPULATE_WRITE = 23
hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
torch.cuda.init()
res = {"GiB": SIZE / G, "busy_GiB": BUSY, "cpus": len(os.sched_getaffinity(0))}
stop = threading.Event()
hold = None
if BUSY > 0:  # the trainer's situation: most of HBM allocated, kernels running on the device
    hold = torch.empty(int(BUSY * G), dtype=torch.uint8, device="cuda")
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)

    def spin():
        while not stop.is_set():
            for _ in range(20):
                a @ a
            torch.cuda.synchronize()
    threading.Thread(target=spin, daemon=True).start()


def gbps(dt):
    return round(SIZE / dt / 1e9, 1) if dt > 0 else None


def case(name):
    kind = name.rstrip("0123456789")
    nth = int(name[len(kind):] or 1)
    path = f"/dev/shm/dlgm-popbench-{name}"
    fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o600)
    os.ftruncate(fd, SIZE)
    m = mmap.mmap(fd, SIZE, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
    buf = ctypes.c_char.from_buffer(m)
    addr = ctypes.addressof(buf)
    pieces = list(range(0, SIZE, G))
    t0 = time.time()
    if kind == "falloc":
        with ThreadPoolExecutor(nth) as ex:
            list(ex.map(lambda off: os.posix_fallocate(fd, off, G), pieces))
        res[name + "_falloc_GBps"] = gbps(time.time() - t0)
        t1 = time.time()
        a8 = np.frombuffer(m, dtype=np.uint8)
        with ThreadPoolExecutor(nth) as ex:
            list(ex.map(lambda off: int(a8[off:off + G:4096].sum()), pieces))
        del a8
        res[name + "_map_GBps"] = gbps(time.time() - t1)
    elif kind == "freg":
        with ThreadPoolExecutor(nth) as ex:
            list(ex.map(lambda off: os.posix_fallocate(fd, off, G), pieces))
    elif kind in ("popw", "huge"):
        if kind == "huge":
            res[name + "_madv_huge_rc"] = libc.madvise(addr, SIZE, 14)
        rcs = []
        with ThreadPoolExecutor(nth) as ex:
            rcs = list(ex.map(lambda off: libc.madvise(addr + off, G, MADV_POPULATE_WRITE), pieces))
        res[name + "_rc"] = max(rcs)
    elif kind == "touch":
        a8 = np.frombuffer(m, dtype=np.uint8)

        def touch(off):
            a8[off:off + G:4096] = 0
        with ThreadPoolExecutor(nth) as ex:
            list(ex.map(touch, pieces))
        del a8
    res[name + "_ready_GBps"] = gbps(time.time() - t0)
    os.close(fd)
    t = time.time()
    regs = []
    for off in pieces:
        if hip.hipHostRegister(addr + off, G, 0) != 0:
            res[name + "_reg_error"] = off
            break
        regs.append(addr + off)
    res[name + "_register_GBps"] = gbps(time.time() - t)
    res[name + "_total_GBps"] = gbps(time.time() - t0)
    for r in regs:
        hip.hipHostUnregister(r)
    del buf
    m.close()
    os.unlink(path)
    print(name, json.dumps({k: v for k, v in res.items() if k.startswith(name + "_")}), flush=True)


for c in os.environ.get("CASES", "falloc1,falloc8,popw1,popw4,popw8,popw16,touch8").split(","):
    case(c)
stop.set()
time.sleep(0.5)  # let the device loop see the stop before the interpreter exits
os.makedirs("gpurun_out/digest", exist_ok=True)
with open(f"gpurun_out/digest/populate_bench_busy{int(BUSY)}.json", "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps(res))
