"""Round 5: what makes a fresh /dev/shm snapshot file ready for DMA fastest on the GPU box? The emergency checkpoint
of an unprepared 81.7 GB snapshot ran at 5 GB/s whether the pages were written through the mapping or page-locked
(hipHostRegister), while a registration of pages a restore had just READ through the mapping ran at ~60 GB/s.
Cases (SIZE GiB each, 1 GiB register pieces):
  reg_fresh      register a sparse file's mapping (allocation + zeroing + mapping inside the registration)
  reg_falloc     fallocate, then register
  read_falloc    fallocate, then read one byte per 4 KiB page through the mapping (read faults map 16 pages)
  reg_after_read ... then register
  popr_falloc    fallocate, then MADV_POPULATE_READ, then register"""
import ctypes
import json
import mmap
import os
import time

import torch

G = 1 << 30
SIZE = int(float(os.environ.get("SIZE", "24")) * G)
libc = ctypes.CDLL("libc.so.6", use_errno=True)
libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
MADV_POPULATE_READ = 22
hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
torch.cuda.init()
res = {"GiB": SIZE / G}


def gbps(dt):
    return round(SIZE / dt / 1e9, 1) if dt > 0 else None


def case(name, falloc, read, popr, mt_read=False):
    path = f"/dev/shm/dlgm-mapbench-{name}"
    fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o600)
    os.ftruncate(fd, SIZE)
    if falloc:
        t = time.time()
        os.posix_fallocate(fd, 0, SIZE)
        res[name + "_falloc_GBps"] = gbps(time.time() - t)
    m = mmap.mmap(fd, SIZE, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
    os.close(fd)
    buf = ctypes.c_char.from_buffer(m)
    addr = ctypes.addressof(buf)
    if read:
        t = time.time()
        a = torch.frombuffer(m, dtype=torch.uint8)
        s = int(a[::4096].sum())  # one byte per page
        res[name + "_read_GBps"] = gbps(time.time() - t)
        del a
    if mt_read:  # read pass on the C++ host runtime's threads (the CRC of every 64 MiB chunk)
        import sys
        sys.path.insert(0, ".")
        from distributed_llm_training_gpu_manager_amd import _host
        t = time.time()
        _host.crc32c_chunks(torch.frombuffer(m, dtype=torch.uint8))
        res[name + "_mt_read_GBps"] = gbps(time.time() - t)
        res[name + "_threads"] = _host.THREADS
    if popr:
        t = time.time()
        rc = libc.madvise(addr, SIZE, MADV_POPULATE_READ)
        res[name + "_populate_read_GBps"] = gbps(time.time() - t)
        res[name + "_populate_rc"] = rc
    t = time.time()
    regs = []
    for off in range(0, SIZE, G):
        if hip.hipHostRegister(addr + off, G, 0) != 0:
            res[name + "_reg_error"] = off
            break
        regs.append(addr + off)
    res[name + "_register_GBps"] = gbps(time.time() - t)
    for r in regs:
        hip.hipHostUnregister(r)
    del buf
    m.close()
    os.unlink(path)
    print(name, json.dumps({k: v for k, v in res.items() if k.startswith(name)}), flush=True)


for c in os.environ.get("CASES", "reg_fresh,reg_falloc,read_falloc,popr_falloc,mtread_falloc").split(","):
    case(c, c != "reg_fresh", c == "read_falloc", c == "popr_falloc", c == "mtread_falloc")
os.makedirs("gpurun_out/digest", exist_ok=True)
with open("gpurun_out/digest/map_bench.json", "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps(res))
