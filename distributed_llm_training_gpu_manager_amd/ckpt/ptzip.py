"""Streaming writer/reader of torch-zip ``.pt`` files whose tensor data is written by the C++ host runtime.

DeepSpeed keeps checkpoints as ``torch.save`` files (``zero_pp_rank_{r}_mp_rank_00_
{model,optim}_states.pt``; the reference asks for them through ``stage3_gather_16bit_weights_on_model_save``,
``ai_engine/deepspeed_launcher.py:74, :192``). ``torch.save`` itself serialises one tensor at a time on
one thread from memory the caller must already hold. A rank of a 70B ZeRO-3 job writes 141 GB, so this
module produces the SAME file format without that constraint:

* the pickle (``archive/data.pkl``) is generated up front from a structure whose large tensors are
  :class:`Slot` placeholders (dtype + shape), with the exact opcodes ``torch.save`` emits
  (``torch._utils._rebuild_tensor_v2`` + typed storages), so ``torch.load(weights_only=True)`` -- and
  ``mmap=True`` -- read it;
* the zip container is laid out by hand: stored (uncompressed) records, ZIP64 sizes and offsets, and
  every record's data 64-byte aligned (``archive/.storage_alignment``), like torch's own writer;
* each slot's bytes are then written at their file offset, in pieces, from pinned staging buffers by
  ``dlgm_pwrite_at2`` (8 threads, CRC32C per 64 MiB chunk for our manifests and the zip CRC-32 for the
  record header, combined with zlib's ``crc32_combine``) -- the file is a valid zip (``unzip -t`` clean).
"""
from __future__ import annotations

import collections
import ctypes
import io
import os
import pickle
import struct
import zlib
from typing import Any, Dict, List, Optional, Tuple

import torch

from .. import _host

ALIGN = 64
_STORAGE = {torch.float32: torch.FloatStorage, torch.bfloat16: torch.BFloat16Storage,
            torch.float16: torch.HalfStorage, torch.int64: torch.LongStorage, torch.int32: torch.IntStorage,
            torch.uint8: torch.ByteStorage, torch.float64: torch.DoubleStorage}


class _StorageRef:
    def __init__(self, key: str, dtype: torch.dtype, numel: int):
        self.key, self.dtype, self.numel = key, dtype, numel


class Slot:
    """A tensor whose bytes are written later (``PtWriter.write``) -- a placeholder inside the saved object."""

    def __init__(self, name: str, dtype: torch.dtype, shape: Tuple[int, ...]):
        self.name, self.dtype, self.shape = name, dtype, tuple(int(s) for s in shape)
        self.numel = 1
        for s in self.shape:
            self.numel *= s
        self.nbytes = self.numel * torch.empty((), dtype=dtype).element_size()
        self.ref: Optional[_StorageRef] = None

    def __reduce_ex__(self, proto):
        stride, acc = [], 1
        for s in reversed(self.shape):
            stride.append(acc)
            acc *= s
        return (torch._utils._rebuild_tensor_v2,
                (self.ref, 0, self.shape, tuple(reversed(stride)), False, collections.OrderedDict()))


class _Pickler(pickle.Pickler):
    def persistent_id(self, obj):
        if isinstance(obj, _StorageRef):
            return ("storage", _STORAGE[obj.dtype], obj.key, "cpu", obj.numel)
        return None


def _inline_tensors(obj, inline: Dict[str, torch.Tensor], slots: List[Slot]):
    """Replace real CPU tensors by slots carrying their bytes inline (small metadata tensors)."""
    if isinstance(obj, torch.Tensor):
        t = obj.detach().cpu().contiguous()
        s = Slot(f"_inline{len(inline)}", t.dtype, tuple(t.shape))
        inline[s.name] = t
        slots.append(s)
        return s
    if isinstance(obj, Slot):
        slots.append(obj)
        return obj
    if isinstance(obj, dict):
        return type(obj)((k, _inline_tensors(v, inline, slots)) for k, v in obj.items()) \
            if not isinstance(obj, collections.OrderedDict) else \
            collections.OrderedDict((k, _inline_tensors(v, inline, slots)) for k, v in obj.items())
    if isinstance(obj, (list, tuple)):
        out = [_inline_tensors(v, inline, slots) for v in obj]
        return out if isinstance(obj, list) else tuple(out)
    return obj


class PtWriter:
    """Lay out a torch-zip file for `obj` (nested dicts/lists with Slots / small tensors), then stream slots."""

    def __init__(self, path: str, obj: Any, prefix: str = "archive"):
        self.path = path
        inline: Dict[str, torch.Tensor] = {}
        slots: List[Slot] = []
        obj = _inline_tensors(obj, inline, slots)
        seen = set()
        self.slots: Dict[str, Slot] = {}
        for i, s in enumerate(slots):
            assert s.name not in seen, f"duplicate slot {s.name}"
            seen.add(s.name)
            s.ref = _StorageRef(str(i), s.dtype, s.numel)
            self.slots[s.name] = s
        buf = io.BytesIO()
        _Pickler(buf, protocol=2).dump(obj)
        records: List[Tuple[str, Any]] = [("data.pkl", buf.getvalue()), (".format_version", b"1"),
                                          (".storage_alignment", str(ALIGN).encode()), ("byteorder", b"little")]
        for s in slots:
            records.append((f"data/{s.ref.key}", s))
        records.append(("version", b"3\n"))
        records.append((".data/serialization_id", str(abs(hash(path)) % 10 ** 20).zfill(40).encode()))
        self._entries = []  # (name, header_off, data_off, size, crc or None, slot)
        off = 0
        headers: List[Tuple[int, bytes]] = []
        small: List[Tuple[int, bytes]] = []
        for name, data in records:
            fname = f"{prefix}/{name}".encode()
            size = data.nbytes if isinstance(data, Slot) else len(data)
            base = off + 30 + len(fname) + 20
            pad = (-base) % ALIGN
            if 0 < pad < 4:
                pad += ALIGN
            extra = struct.pack("<HHQQ", 0x0001, 16, size, size)
            if pad:
                extra += struct.pack("<HH", 0x4246, pad - 4) + b"\0" * (pad - 4)
            crc = 0 if isinstance(data, Slot) else zlib.crc32(data) & 0xFFFFFFFF
            hdr = struct.pack("<IHHHHHIIIHH", 0x04034B50, 45, 0, 0, 0, 0x21, crc, 0xFFFFFFFF, 0xFFFFFFFF,
                              len(fname), len(extra)) + fname + extra
            data_off = off + len(hdr)
            assert data_off % ALIGN == 0
            headers.append((off, hdr))
            if not isinstance(data, Slot):
                small.append((data_off, data))
            self._entries.append([fname, off, data_off, size, None if isinstance(data, Slot) else crc,
                                  data if isinstance(data, Slot) else None])
            if isinstance(data, Slot):
                data.file_off = data_off
            off = data_off + size
        self.cd_off = off
        self._crc_parts: Dict[str, List[Tuple[int, int, int]]] = {s.name: [] for s in slots}  # (rel_off, len, crc)
        L = _host.lib()
        fd = L.dlgm_open_write(path.encode(), 0) if L is not None else -1
        if L is not None and fd < 0:
            raise OSError(-fd, os.strerror(-fd), path)
        self._fd = fd if L is not None else os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        for o, h in headers + small:
            os.pwrite(self._fd, h, o)
        self.chunk_crcs: Dict[str, List[int]] = {s.name: [0] * max(1, (s.nbytes + _host.CHUNK - 1) // _host.CHUNK)
                                                 for s in slots}
        for name, t in inline.items():
            self.write(name, t, 0)

    def write(self, name: str, t: torch.Tensor, rel_off: int) -> None:
        """Write the bytes of contiguous CPU tensor `t` at byte `rel_off` of slot `name` (a CHUNK multiple)."""
        s = self.slots[name]
        assert t.device.type == "cpu" and t.is_contiguous() and rel_off % _host.CHUNK == 0
        n = t.numel() * t.element_size()
        assert rel_off + n <= s.nbytes, (name, rel_off, n, s.nbytes)
        if n == 0:
            return
        nch = (n + _host.CHUNK - 1) // _host.CHUNK
        L = _host.lib()
        first = rel_off // _host.CHUNK
        if L is not None:
            crcs = (ctypes.c_uint32 * nch)()
            zcrcs = (ctypes.c_uint32 * nch)()
            rc = L.dlgm_pwrite_at2(self._fd, ctypes.c_void_p(t.data_ptr()), n, s.file_off + rel_off, _host.CHUNK,
                                   _host.THREADS, crcs, zcrcs)
            if rc != 0:
                raise OSError(-rc, os.strerror(-rc), self.path)
            self.chunk_crcs[name][first:first + nch] = list(crcs)
            for i in range(nch):
                ln = min(_host.CHUNK, n - i * _host.CHUNK)
                self._crc_parts[name].append((rel_off + i * _host.CHUNK, ln, zcrcs[i]))
        else:
            mv = memoryview(t.view(torch.uint8).numpy())
            os.pwrite(self._fd, mv, s.file_off + rel_off)
            for i in range(nch):
                piece = mv[i * _host.CHUNK:(i + 1) * _host.CHUNK]
                self.chunk_crcs[name][first + i] = zlib.crc32(piece) & 0xFFFFFFFF
                self._crc_parts[name].append((rel_off + i * _host.CHUNK, len(piece), zlib.crc32(piece) & 0xFFFFFFFF))

    def _slot_crc(self, name: str) -> int:
        parts = sorted(self._crc_parts[name])
        s = self.slots[name]
        covered = sum(p[1] for p in parts)
        if covered != s.nbytes:
            raise RuntimeError(f"{self.path}: slot {name} written {covered} of {s.nbytes} bytes")
        L = _host.lib()
        crc = 0
        for _, ln, c in parts:
            if L is not None:
                crc = L.dlgm_crc32_combine(crc, c, ln)
            else:
                crc = _crc32_combine_py(crc, c, ln)
        return crc

    def close(self, fsync: bool = True) -> Dict[str, Dict[str, Any]]:
        """Patch the record CRCs, write the central directory; returns {slot: {offset, bytes, crc32c chunks}}."""
        cd = b""
        for ent in self._entries:
            fname, hoff, doff, size, crc, slot = ent
            if slot is not None:
                crc = self._slot_crc(slot.name)
                os.pwrite(self._fd, struct.pack("<I", crc), hoff + 14)
            extra = struct.pack("<HHQQQ", 0x0001, 24, size, size, hoff)
            cd += struct.pack("<IHHHHHHIIIHHHHHII", 0x02014B50, 45, 45, 0, 0, 0, 0x21, crc, 0xFFFFFFFF,
                              0xFFFFFFFF, len(fname), len(extra), 0, 0, 0, 0, 0xFFFFFFFF) + fname + extra
        n = len(self._entries)
        z64 = self.cd_off + len(cd)
        tail = struct.pack("<IQHHIIQQQQ", 0x06064B50, 44, 45, 45, 0, 0, n, n, len(cd), self.cd_off)
        tail += struct.pack("<IIQI", 0x07064B50, 0, z64, 1)
        tail += struct.pack("<IHHHHIIH", 0x06054B50, 0, 0, 0xFFFF, 0xFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0)
        os.pwrite(self._fd, cd + tail, self.cd_off)
        L = _host.lib()
        if L is not None:
            rc = L.dlgm_close_file(self._fd, int(fsync))
            if rc != 0:
                raise OSError(-rc, os.strerror(-rc), self.path)
        else:
            if fsync:
                os.fsync(self._fd)
            os.close(self._fd)
        return {name: {"offset": s.file_off, "bytes": s.nbytes, "crc": self.chunk_crcs[name],
                       "chunk": _host.CHUNK, "algo": _host.algo() if _host.lib() is not None else "crc32-zlib"}
                for name, s in self.slots.items() if not name.startswith("_inline")}


def _crc32_combine_py(crc1: int, crc2: int, len2: int) -> int:
    """zlib crc32_combine in Python (only without the host library)."""
    def gf2_times(mat, vec):
        s, i = 0, 0
        while vec:
            if vec & 1:
                s ^= mat[i]
            vec >>= 1
            i += 1
        return s

    def gf2_square(mat):
        return [gf2_times(mat, mat[n]) for n in range(32)]
    if len2 <= 0:
        return crc1
    odd = [0xEDB88320] + [1 << n for n in range(31)]
    even = gf2_square(odd)
    odd = gf2_square(even)
    while True:
        even = gf2_square(odd)
        if len2 & 1:
            crc1 = gf2_times(even, crc1)
        len2 >>= 1
        if not len2:
            break
        odd = gf2_square(even)
        if len2 & 1:
            crc1 = gf2_times(odd, crc1)
        len2 >>= 1
        if not len2:
            break
    return crc1 ^ crc2


def record_offsets(path: str) -> Dict[str, Tuple[int, int]]:
    """{record name without the archive prefix: (data offset, size)} of a stored torch-zip file."""
    with open(path, "rb") as f:
        f.seek(0, 2)
        end = f.tell()
        f.seek(max(0, end - 65536 - 22))
        tail = f.read()
        i = tail.rfind(b"PK\x05\x06")
        if i < 0:
            raise ValueError(f"{path}: not a zip file")
        _, _, _, n16, _, cd_size, cd_off, _ = struct.unpack("<IHHHHIIH", tail[i:i + 22])
        if cd_off == 0xFFFFFFFF or n16 == 0xFFFF:
            j = tail.rfind(b"PK\x06\x06")
            rec = struct.unpack("<IQHHIIQQQQ", tail[j:j + 56])
            cd_size, cd_off = rec[8], rec[9]
        f.seek(cd_off)
        cd = f.read(cd_size)
        out: Dict[str, Tuple[int, int]] = {}
        p = 0
        while p + 46 <= len(cd) and cd[p:p + 4] == b"PK\x01\x02":
            (_, _, _, _, method, _, _, _, csize, usize, nlen, xlen, clen, _, _, _, hoff) = \
                struct.unpack("<IHHHHHHIIIHHHHHII", cd[p:p + 46])
            name = cd[p + 46:p + 46 + nlen].decode()
            extra = cd[p + 46 + nlen:p + 46 + nlen + xlen]
            q = 0
            while q + 4 <= len(extra):
                hid, hsz = struct.unpack("<HH", extra[q:q + 4])
                if hid == 0x0001:
                    vals = list(struct.unpack("<" + "Q" * (hsz // 8), extra[q + 4:q + 4 + hsz]))
                    if usize == 0xFFFFFFFF:
                        usize = vals.pop(0)
                    if csize == 0xFFFFFFFF:
                        csize = vals.pop(0)
                    if hoff == 0xFFFFFFFF:
                        hoff = vals.pop(0)
                q += 4 + hsz
            f.seek(hoff)
            lh = f.read(30)
            lnlen, lxlen = struct.unpack("<HH", lh[26:30])
            if method != 0:
                raise ValueError(f"{path}: record {name} is compressed")
            out[name.split("/", 1)[1] if "/" in name else name] = (hoff + 30 + lnlen + lxlen, usize)
            p += 46 + nlen + xlen + clen
    return out


def read_slot(path: str, t: torch.Tensor, file_off: int) -> List[int]:
    """Fill contiguous CPU tensor `t` from `path` at `file_off`; per-chunk CRC32C (C++, 8 threads)."""
    n = t.numel() * t.element_size()
    nch = (n + _host.CHUNK - 1) // _host.CHUNK
    L = _host.lib()
    if L is not None:
        crcs = (ctypes.c_uint32 * max(nch, 1))()
        rc = L.dlgm_read_file_at(path.encode(), ctypes.c_void_p(t.data_ptr()), n, file_off, _host.CHUNK,
                                 _host.THREADS, crcs)
        if rc != 0:
            raise OSError(-rc, os.strerror(-rc), path)
        return list(crcs)[:nch]
    mv = memoryview(t.view(torch.uint8).numpy())
    with open(path, "rb") as f:
        f.seek(file_off)
        f.readinto(mv)
    return [zlib.crc32(mv[i * _host.CHUNK:(i + 1) * _host.CHUNK]) & 0xFFFFFFFF for i in range(nch)]
