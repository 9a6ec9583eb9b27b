"""ctypes binding of the host runtime ``_dlgm_host.so`` (csrc/host): checkpoint file I/O with
CRC32C, and the AVX2 CPU AdamW used by the ZeRO-Offload path. Falls back to Python (zlib /
torch) only if the library was not built, and says so in the manifest ("crc" algorithm name)."""
from __future__ import annotations

import ctypes
import os
import zlib
from typing import List, Optional, Tuple

import numpy as np
import torch

from ._native import HOST_LIB

_lib = None


def lib():
    global _lib
    if _lib is None and HOST_LIB.exists():
        L = ctypes.CDLL(str(HOST_LIB))
        L.dlgm_crc32c.restype = ctypes.c_uint32
        L.dlgm_crc32c.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32]
        for fn in (L.dlgm_write_file, L.dlgm_read_file):
            fn.restype = ctypes.c_int
        L.dlgm_write_file.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                      ctypes.c_int, ctypes.POINTER(ctypes.c_uint32), ctypes.c_int]
        L.dlgm_read_file.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                     ctypes.c_int, ctypes.POINTER(ctypes.c_uint32)]
        L.dlgm_open_write.restype = ctypes.c_int
        L.dlgm_open_write.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.dlgm_pwrite_at.restype = ctypes.c_int
        L.dlgm_pwrite_at.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                     ctypes.c_int, ctypes.POINTER(ctypes.c_uint32)]
        L.dlgm_close_file.restype = ctypes.c_int
        L.dlgm_close_file.argtypes = [ctypes.c_int, ctypes.c_int]
        L.dlgm_cpu_adamw.restype = None
        L.dlgm_cpu_adamw.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t] + [ctypes.c_float] * 8
        _lib = L
    return _lib


CHUNK = 64 << 20
THREADS = int(os.environ.get("DLGM_CKPT_THREADS", "8"))


def algo() -> str:
    return "crc32c" if lib() is not None else "crc32-zlib"


def _crc_py(buf: memoryview) -> int:
    return zlib.crc32(buf) & 0xFFFFFFFF


def write_tensor(path: str, t: torch.Tensor, fsync: bool = True) -> List[int]:
    """Write a contiguous CPU tensor's bytes to `path`; return per-64 MiB-chunk checksums."""
    assert t.device.type == "cpu" and t.is_contiguous()
    n = t.numel() * t.element_size()
    nch = (n + CHUNK - 1) // CHUNK
    L = lib()
    if L is not None:
        crcs = (ctypes.c_uint32 * max(nch, 1))()
        rc = L.dlgm_write_file(path.encode(), ctypes.c_void_p(t.data_ptr()), n, CHUNK, THREADS, crcs, int(fsync))
        if rc != 0:
            raise OSError(-rc, os.strerror(-rc), path)
        return list(crcs)[:nch]
    mv = memoryview(t.view(torch.uint8).numpy()) if n else memoryview(b"")
    with open(path, "wb") as f:
        f.write(mv)
        if fsync:
            f.flush()
            os.fsync(f.fileno())
    return [_crc_py(mv[i * CHUNK:(i + 1) * CHUNK]) for i in range(nch)]


def read_tensor(path: str, t: torch.Tensor) -> List[int]:
    """Fill a contiguous CPU tensor from `path`; return per-chunk checksums (for verification)."""
    assert t.device.type == "cpu" and t.is_contiguous()
    n = t.numel() * t.element_size()
    nch = (n + CHUNK - 1) // CHUNK
    L = lib()
    if L is not None:
        crcs = (ctypes.c_uint32 * max(nch, 1))()
        rc = L.dlgm_read_file(path.encode(), ctypes.c_void_p(t.data_ptr()), n, CHUNK, THREADS, crcs)
        if rc != 0:
            raise OSError(-rc, os.strerror(-rc), path)
        return list(crcs)[:nch]
    arr = t.view(torch.uint8).numpy()
    with open(path, "rb") as f:
        f.readinto(memoryview(arr))
    mv = memoryview(arr)
    return [_crc_py(mv[i * CHUNK:(i + 1) * CHUNK]) for i in range(nch)]


def cpu_adamw_(p, m, v, g, p16, lr, b1, b2, eps, wd, bc1, bc2, gscale=1.0) -> None:
    L = lib()
    if L is None:
        raise RuntimeError("host runtime _dlgm_host.so not built")
    for t in (p, m, v, g):
        assert t.device.type == "cpu" and t.dtype == torch.float32 and t.is_contiguous()
    L.dlgm_cpu_adamw(p.data_ptr(), m.data_ptr(), v.data_ptr(), g.data_ptr(),
                     p16.data_ptr() if p16 is not None else None, p.numel(), lr, b1, b2, eps, wd, bc1, bc2, gscale)


class StreamWriter:
    """Write one file from chunk-aligned pieces (pinned ring slots) at their offsets."""

    def __init__(self, path: str, total: int):
        self.path, self.total = path, total
        self.crcs: List[int] = [0] * ((total + CHUNK - 1) // CHUNK)
        L = lib()
        if L is not None:
            fd = L.dlgm_open_write(path.encode(), total)
            if fd < 0:
                raise OSError(-fd, os.strerror(-fd), path)
            self.fd, self.f = fd, None
        else:
            self.fd, self.f = -1, open(path, "wb")
            self.f.truncate(total)

    def write(self, t: torch.Tensor, offset: int) -> None:
        assert offset % CHUNK == 0 and t.is_contiguous() and t.device.type == "cpu"
        n = t.numel() * t.element_size()
        nch = (n + CHUNK - 1) // CHUNK
        first = offset // CHUNK
        L = lib()
        if L is not None:
            crcs = (ctypes.c_uint32 * max(nch, 1))()
            rc = L.dlgm_pwrite_at(self.fd, ctypes.c_void_p(t.data_ptr()), n, offset, CHUNK, THREADS, crcs)
            if rc != 0:
                raise OSError(-rc, os.strerror(-rc), self.path)
            self.crcs[first:first + nch] = list(crcs)[:nch]
        else:
            mv = memoryview(t.view(torch.uint8).numpy())
            self.f.seek(offset)
            self.f.write(mv)
            self.crcs[first:first + nch] = [_crc_py(mv[i * CHUNK:(i + 1) * CHUNK]) for i in range(nch)]

    def close(self, fsync: bool = True) -> List[int]:
        L = lib()
        if L is not None:
            rc = L.dlgm_close_file(self.fd, int(fsync))
            if rc != 0:
                raise OSError(-rc, os.strerror(-rc), self.path)
        else:
            self.f.flush()
            if fsync:
                os.fsync(self.f.fileno())
            self.f.close()
        return self.crcs
