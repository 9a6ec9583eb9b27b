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
        L.dlgm_read_file_at.restype = ctypes.c_int
        L.dlgm_read_file_at.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                        ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_uint32)]
        L.dlgm_pwrite_at2.restype = ctypes.c_int
        L.dlgm_pwrite_at2.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                      ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_uint32),
                                      ctypes.POINTER(ctypes.c_uint32)]
        L.dlgm_crc32_combine.restype = ctypes.c_uint32
        L.dlgm_crc32_combine.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]
        L.dlgm_crc32_zip.restype = ctypes.c_uint32
        L.dlgm_crc32_zip.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        L.dlgm_crc32c_chunks.restype = None
        L.dlgm_crc32c_chunks.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_uint32)]
        L.dlgm_copy_crc32c_chunks.restype = None
        L.dlgm_copy_crc32c_chunks.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                              ctypes.c_int, ctypes.POINTER(ctypes.c_uint32)]
        L.dlgm_touch_pages.restype = ctypes.c_uint64
        L.dlgm_touch_pages.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        if hasattr(L, "dlgm_populate_pages"):
            L.dlgm_populate_pages.restype = ctypes.c_int
            L.dlgm_populate_pages.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int]
        L.dlgm_close_file.restype = ctypes.c_int
        L.dlgm_close_file.argtypes = [ctypes.c_int, ctypes.c_int]
        L.dlgm_aio_create.restype = ctypes.c_void_p
        L.dlgm_aio_create.argtypes = [ctypes.c_int, ctypes.c_size_t]
        L.dlgm_aio_destroy.restype = None
        L.dlgm_aio_destroy.argtypes = [ctypes.c_void_p]
        L.dlgm_aio_open.restype = ctypes.c_int
        L.dlgm_aio_open.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_size_t]
        L.dlgm_aio_is_direct.restype = ctypes.c_int
        L.dlgm_aio_is_direct.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.dlgm_aio_close.restype = ctypes.c_int
        L.dlgm_aio_close.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.dlgm_aio_submit.restype = ctypes.c_int64
        L.dlgm_aio_submit.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                      ctypes.c_int]
        for fn in (L.dlgm_aio_wait, L.dlgm_aio_poll):
            fn.restype = ctypes.c_int
            fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        L.dlgm_cpu_adamw.restype = None
        L.dlgm_cpu_adamw.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t] + [ctypes.c_float] * 8
        _lib = L
    return _lib


CHUNK = 64 << 20
# checkpoint I/O + CRC threads: 16 = the CPU share of one GPU on an 8-GPU MI355X node
THREADS = max(4, min(16, (os.cpu_count() or 8) // 2))  # checkpoint I/O / CRC threads


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


def crc32c_chunks(t: torch.Tensor) -> List[int]:
    """Per-CHUNK CRC32C of a contiguous CPU tensor's bytes (8 threads; verifies a /dev/shm snapshot)."""
    n = t.numel() * t.element_size()
    nch = (n + CHUNK - 1) // CHUNK
    L = lib()
    if L is None:
        mv = memoryview(t.view(torch.uint8).numpy())
        return [_crc_py(mv[i * CHUNK:(i + 1) * CHUNK]) for i in range(nch)]
    crcs = (ctypes.c_uint32 * max(nch, 1))()
    L.dlgm_crc32c_chunks(ctypes.c_void_p(t.data_ptr()), n, CHUNK, THREADS, crcs)
    return list(crcs)[:nch]


def copy_crc32c_chunks(src: torch.Tensor, dst: torch.Tensor) -> List[int]:
    """dst <- src (contiguous CPU byte tensors of one size, e.g. a mapped /dev/shm file slice into a pinned
    slot) on THREADS threads, with the per-CHUNK CRC32C of the copied bytes."""
    n = src.numel() * src.element_size()
    assert dst.numel() * dst.element_size() == n and src.is_contiguous() and dst.is_contiguous()
    nch = (n + CHUNK - 1) // CHUNK
    L = lib()
    if L is None:
        dst.view(torch.uint8).copy_(src.view(torch.uint8))
        return crc32c_chunks(dst)
    crcs = (ctypes.c_uint32 * max(nch, 1))()
    L.dlgm_copy_crc32c_chunks(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()), n, CHUNK, THREADS,
                              crcs)
    return list(crcs)[:nch]


def touch_pages(t: torch.Tensor, threads: int = THREADS) -> int:
    """Read one byte per 4 KiB page of a contiguous CPU tensor (a mapped /dev/shm file) on `threads` threads:
    maps the pages into this process, zeroing reserved-but-untouched tmpfs pages on the way. Returns the byte sum."""
    n = t.numel() * t.element_size()
    L = lib()
    if L is None:
        return int(t.view(torch.uint8)[::4096].sum()) if n else 0
    return int(L.dlgm_touch_pages(ctypes.c_void_p(t.data_ptr()), n, int(threads)))


def populate_pages(t: torch.Tensor, threads: int = 16, write: bool = True) -> bool:
    """Map the pages of a contiguous CPU tensor (a mapped /dev/shm file) into this process with MADV_POPULATE_WRITE
    (or _READ) on `threads` threads (csrc/host/ckpt_io.cpp: 64 GB/s on the MI355X host, and the page-lock after a
    populate-write 3x faster than after a read touch). False when unavailable (old kernel, library not built): the
    caller touches the pages instead."""
    L = lib()
    n = t.numel() * t.element_size()
    if L is None or not hasattr(L, "dlgm_populate_pages") or n == 0:
        return False
    return int(L.dlgm_populate_pages(ctypes.c_void_p(t.data_ptr()), n, int(threads), int(bool(write)))) == 0


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


def aligned_empty(numel: int, dtype: torch.dtype = torch.float32, align: int = 4096) -> torch.Tensor:
    """A CPU tensor whose storage starts on an `align`-byte boundary (O_DIRECT staging)."""
    esz = torch.empty((), dtype=dtype).element_size()
    raw = torch.empty(numel * esz + align, dtype=torch.uint8)
    skip = (-raw.data_ptr()) % align
    return raw[skip:skip + numel * esz].view(dtype)


class Aio:
    """Asynchronous pread/pwrite engine (csrc/host/aio.cpp): a persistent I/O thread pool, requests split
    into `block_size` pieces, non-blocking submit returning a ticket. DeepSpeed ``aio`` block parity:
    ``thread_count`` x ``queue_depth`` pieces in flight."""

    def __init__(self, threads: int = 8, block_size: int = 8 << 20):
        L = lib()
        if L is None:
            raise RuntimeError("host runtime _dlgm_host.so not built")
        self._L = L
        self._e = ctypes.c_void_p(L.dlgm_aio_create(int(threads), int(block_size)))

    def open(self, path: str, size: int = 0, direct: bool = False) -> int:
        h = self._L.dlgm_aio_open(self._e, path.encode(), int(direct), int(size))
        if h < 0:
            raise OSError(-h, os.strerror(-h), path)
        return h

    def is_direct(self, h: int) -> bool:
        return bool(self._L.dlgm_aio_is_direct(self._e, h))

    def _submit(self, h: int, t: torch.Tensor, offset: int, write: int) -> int:
        assert t.device.type == "cpu" and t.is_contiguous()
        tk = self._L.dlgm_aio_submit(self._e, h, ctypes.c_void_p(t.data_ptr()), t.numel() * t.element_size(),
                                     int(offset), write)
        if tk < 0:
            raise OSError(-tk, os.strerror(-tk))
        return tk

    def read(self, h: int, t: torch.Tensor, offset: int) -> int:
        """Start filling `t` from byte `offset` of file `h`; returns a ticket (keep `t` alive until waited)."""
        return self._submit(h, t, offset, 0)

    def write(self, h: int, t: torch.Tensor, offset: int) -> int:
        return self._submit(h, t, offset, 1)

    def wait(self, ticket: int) -> None:
        rc = self._L.dlgm_aio_wait(self._e, ticket)
        if rc != 0:
            raise OSError(-rc, os.strerror(-rc))

    def done(self, ticket: int) -> bool:
        return self._L.dlgm_aio_poll(self._e, ticket) == 1

    def close(self, h: int, fsync: bool = False) -> None:
        rc = self._L.dlgm_aio_close(self._e, h, int(fsync))
        if rc != 0:
            raise OSError(-rc, os.strerror(-rc))

    def shutdown(self) -> None:
        if self._e:
            self._L.dlgm_aio_destroy(self._e)  # drains queued pieces, joins the threads, closes files
            self._e = ctypes.c_void_p(None)

    def __del__(self):
        try:
            self.shutdown()
        except Exception:
            pass
