"""Where the /dev/shm restore time goes: C++ pread+CRC32C into pinned memory, H2D, and the two overlapped."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_llm_training_gpu_manager_amd import _host  # noqa: E402
from distributed_llm_training_gpu_manager_amd.ckpt.ptzip import read_slot  # noqa: E402

GB = 1 << 30
size = int(sys.argv[1]) * GB if len(sys.argv) > 1 else 16 * GB
piece = int(sys.argv[2]) << 20 if len(sys.argv) > 2 else 256 << 20
path = "/dev/shm/dlgm-probe-restore.bin"
res = {"file_GiB": size / GB, "piece_MiB": piece >> 20, "threads": _host.THREADS}
try:
    src = torch.empty(piece, dtype=torch.uint8)
    src.random_(0, 255)
    t0 = time.time()
    with open(path, "wb") as f:
        for off in range(0, size, piece):
            f.write(src.numpy().tobytes())
    res["write_GBps"] = round(size / GB / (time.time() - t0), 2)
    slots = [torch.empty(piece, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    dev = torch.empty(size, dtype=torch.uint8, device="cuda")
    t0 = time.time()
    for i, off in enumerate(range(0, size, piece)):
        read_slot(path, slots[i % 2], off)
    res["read_crc_pinned_GBps"] = round(size / GB / (time.time() - t0), 2)
    torch.cuda.synchronize()
    t0 = time.time()
    for i, off in enumerate(range(0, size, piece)):
        dev[off:off + piece].copy_(slots[i % 2], non_blocking=True)
    torch.cuda.synchronize()
    res["h2d_GBps"] = round(size / GB / (time.time() - t0), 2)
    t0 = time.time()
    L = _host.lib()
    import ctypes
    n = piece
    for i, off in enumerate(range(0, size, piece)):
        crcs = (ctypes.c_uint32 * (n // _host.CHUNK))()
        L.dlgm_crc32c_chunks(ctypes.c_void_p(slots[i % 2].data_ptr()), n, _host.CHUNK, _host.THREADS, crcs)
    res["crc_only_GBps"] = round(size / GB / (time.time() - t0), 2)
    t0 = time.time()
    for i, off in enumerate(range(0, size, piece)):
        with open(path, "rb") as f:
            f.seek(off)
            f.readinto(memoryview(slots[i % 2].numpy()))
    res["python_readinto_GBps"] = round(size / GB / (time.time() - t0), 2)
finally:
    if os.path.exists(path):
        os.unlink(path)
print(json.dumps(res))
