#!/usr/bin/env python3
"""Round 6: mapping a reserved (fallocated) /dev/shm snapshot into the trainer before page-locking it -- one thread
(the round-5 pipeline: 15.6 GB/s, profiles/shm_map_bench_r05.json) vs the native multi-threaded touch (_host.
touch_pages) vs threaded MADV_POPULATE_WRITE; then hipHostRegister of the mapped pages. Each variant on a fresh file."""
import ctypes
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402
from distributed_llm_training_gpu_manager_amd import _host  # noqa: E402

N = int(float(os.environ.get("GIB", "24")) * (1 << 30))
libc = ctypes.CDLL("libc.so.6", use_errno=True)
libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]


def fresh():
    path = "/dev/shm/dlgm-mapbench.snap"
    fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o600)
    os.ftruncate(fd, N)
    t = time.time()
    os.posix_fallocate(fd, 0, N)
    os.close(fd)
    return path, N / (time.time() - t) / 1e9


def popw(snap, nth):
    ptr, chunks = snap.data_ptr(), list(range(0, N, 64 << 20))

    def work(i):
        for off in chunks[i::nth]:
            libc.madvise(ptr + off, min(64 << 20, N - off), 23)
    th = [threading.Thread(target=work, args=(i,)) for i in range(nth)]
    [x.start() for x in th]
    [x.join() for x in th]


def main():
    torch.cuda.init()
    out = {"GiB": N / (1 << 30)}
    variants = [("torch1", lambda s: int(s[::4096].sum())), ("touch4", lambda s: _host.touch_pages(s, 4)),
                ("touch8", lambda s: _host.touch_pages(s, 8)), ("touch16", lambda s: _host.touch_pages(s, 16)),
                ("popw8", lambda s: popw(s, 8)), ("popw16", lambda s: popw(s, 16))]
    for name, fn in variants:
        path, fgb = fresh()
        snap = torch.from_file(path, shared=True, size=N, dtype=torch.uint8)
        t = time.time()
        fn(snap)
        tm = time.time() - t
        t = time.time()
        rc = hip.hipHostRegister(ctypes.c_void_p(snap.data_ptr()), N, 0)
        tr = time.time() - t
        if rc == 0:
            hip.hipHostUnregister(ctypes.c_void_p(snap.data_ptr()))
        out[name] = {"fallocate_GBps": round(fgb, 1), "map_GBps": round(N / tm / 1e9, 1),
                     "register_GBps": round(N / tr / 1e9, 1) if rc == 0 else f"rc={rc}",
                     "map_then_register_GBps": round(N / (tm + tr) / 1e9, 1)}
        print(name, json.dumps(out[name]), flush=True)
        del snap
        os.unlink(path)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
