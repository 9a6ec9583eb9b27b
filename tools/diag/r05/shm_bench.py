"""What does preparing and filling a /dev/shm snapshot cost on the GPU box (an emergency
checkpoint that finds its buffer unprepared took 11.3 s)? Sizes in GiB (SIZE env, default 48):
  fallocate_1t / fallocate_8t : posix_fallocate of the whole file by one thread / by 8 threads on disjoint ranges
  register_s                  : hipHostRegister of the mapping in 1 GiB pieces
  d2h_registered_GBps         : device -> the registered mapping (what a prepared snapshot save does)
  d2h_pageable_GBps           : device -> the fallocated but unregistered mapping (HIP stages it)
  ring_GBps                   : device -> 4 pinned 256 MiB slots -> 16-thread copy (+CRC32C) into the mapping"""
import ctypes
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, ".")
from distributed_llm_training_gpu_manager_amd import _host  # noqa: E402

G = 1 << 30
size = int(float(os.environ.get("SIZE", "48")) * G)
dev = torch.device("cuda", 0)
res = {"GiB": size / G}
lib = ctypes.CDLL("libamdhip64.so")
lib.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
lib.hipHostUnregister.argtypes = [ctypes.c_void_p]


def falloc(path, nthreads):
    fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o600)
    t0 = time.time()
    step = size // nthreads
    ths = [threading.Thread(target=os.posix_fallocate, args=(fd, i * step, size - i * step if i == nthreads - 1
                                                           else step)) for i in range(nthreads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dt = time.time() - t0
    os.close(fd)
    return dt


for nt in (1, 8):
    p = f"/dev/shm/dlgm-bench-{nt}.snap"
    res[f"fallocate_{nt}t_s"] = round(falloc(p, nt), 2)
    if nt == 1:
        os.unlink(p)
path = "/dev/shm/dlgm-bench-8.snap"
snap = torch.from_file(path, shared=True, size=size, dtype=torch.uint8)
src = torch.randint(0, 255, (size,), dtype=torch.uint8, device=dev)
torch.cuda.synchronize()

# unregistered (pageable) D2H into the mapping
t0 = time.time()
snap.copy_(src)
res["d2h_pageable_GBps"] = round(size / (time.time() - t0) / 1e9, 1)

# ring: pinned slots + threaded copy with CRC
slot_b = 256 << 20
slots = [torch.empty(slot_b, dtype=torch.uint8, pin_memory=True) for _ in range(4)]
ev = [None] * 4
stream = torch.cuda.Stream(dev)
t0 = time.time()
pend = []
for k, off in enumerate(range(0, size, slot_b)):
    s = k % 4
    if len(pend) == 4:
        pk, poff, pln = pend.pop(0)
        ev[pk % 4].synchronize()
        _host.copy_crc32c_chunks(slots[pk % 4][:pln], snap[poff:poff + pln])
    ln = min(slot_b, size - off)
    with torch.cuda.stream(stream):
        slots[s][:ln].copy_(src[off:off + ln], non_blocking=True)
        e = torch.cuda.Event()
        e.record(stream)
        ev[s] = e
    pend.append((k, off, ln))
for pk, poff, pln in pend:
    ev[pk % 4].synchronize()
    _host.copy_crc32c_chunks(slots[pk % 4][:pln], snap[poff:poff + pln])
res["ring_GBps"] = round(size / (time.time() - t0) / 1e9, 1)

# register in 1 GiB pieces, then D2H into the registered mapping
t0 = time.time()
regs = []
for off in range(0, size, G):
    ln = min(G, size - off)
    rc = lib.hipHostRegister(snap.data_ptr() + off, ln, 0)
    if rc != 0:
        res["register_error"] = rc
        break
    regs.append(snap.data_ptr() + off)
res["register_s"] = round(time.time() - t0, 2)
torch.cuda.synchronize()
t0 = time.time()
for off in range(0, size, G):
    snap[off:off + G].copy_(src[off:off + G], non_blocking=True)
torch.cuda.synchronize()
res["d2h_registered_GBps"] = round(size / (time.time() - t0) / 1e9, 1)
t0 = time.time()
for r in regs:
    lib.hipHostUnregister(r)
res["unregister_s"] = round(time.time() - t0, 2)
del snap
os.unlink(path)
print(json.dumps(res), flush=True)
os.makedirs("gpurun_out/digest", exist_ok=True)
with open("gpurun_out/digest/shm_bench.json", "w") as f:
    json.dump(res, f, indent=1)
