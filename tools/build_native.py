#!/usr/bin/env python3
"""Build the MI355X-native shared objects in-tree with hipcc (gfx950 only).

Two libraries are produced next to the Python package:

* ``_dlgm_hip.so``  -- the HIP kernels (csrc/kernels/*.hip) + TORCH_LIBRARY
  registrations (csrc/bindings.cpp), loaded with ``torch.ops.load_library``;
* ``_dlgm_host.so`` -- the host runtime (csrc/host/*.cpp): multi-threaded
  checkpoint writer/reader with CRC32C, AVX2/FMA CPU AdamW (ZeRO-Offload). Plain
  C++ built with g++ (no HIP, no torch), driven through ``ctypes``.

We drive hipcc directly instead of ``torch.utils.cpp_extension`` so that no
hipify pass ever touches the sources and the objects are always built for
``--offload-arch=gfx950`` only. Objects are cached under ``build/`` keyed on the
source + header mtimes, so an unchanged tree rebuilds in well under a second.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "distributed_llm_training_gpu_manager_amd"
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "native"
ARCH = "gfx950"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch

    tdir = Path(torch.__file__).resolve().parent
    inc = [tdir / "include", tdir / "include" / "torch" / "csrc" / "api" / "include"]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return tdir / "lib", inc, abi


def _headers_stamp() -> str:
    h = hashlib.sha1()
    for p in sorted((CSRC / "include").glob("*.h")):
        h.update(p.read_bytes())
    return h.hexdigest()[:12]


def _compile(src: Path, obj: Path, flags: list[str], verbose: bool) -> None:
    cmd = [HIPCC, *flags, "-c", str(src), "-o", str(obj)]
    if verbose:
        print(" ".join(cmd), flush=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{res.stdout}\n{res.stderr}")


def _build_lib(name: str, sources: list[Path], cflags: list[str], ldflags: list[str], jobs: int,
               verbose: bool, force: bool) -> Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    stamp = _headers_stamp() + hashlib.sha1(" ".join(cflags).encode()).hexdigest()[:8]
    objs = []
    todo = []
    for src in sources:
        obj = BUILD / f"{src.stem}.{src.suffix[1:]}.{stamp}.o"
        objs.append(obj)
        if force or not obj.exists() or obj.stat().st_mtime < src.stat().st_mtime:
            todo.append((src, obj))
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = [ex.submit(_compile, s, o, cflags, verbose) for s, o in todo]
        for f in futs:
            f.result()
    out = PKG / name
    newest = max((o.stat().st_mtime for o in objs), default=0)
    if force or todo or not out.exists() or out.stat().st_mtime < newest:
        tmp = out.with_suffix(".so.tmp")
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(tmp), *ldflags]
        if verbose:
            print(" ".join(cmd), flush=True)
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed: {name}\n{res.stdout}\n{res.stderr}")
        os.replace(tmp, out)
    return out


def _build_host(sources: list[Path], jobs: int, verbose: bool, force: bool) -> Path:
    """Host runtime: plain C++ (g++, no HIP/torch), -O3 with SSE4.2 CRC32C and AVX2/FMA AdamW."""
    BUILD.mkdir(parents=True, exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    flags = ["-O3", "-std=c++17", "-fPIC", "-fopenmp", "-mavx2", "-mfma", "-Wall", "-Wno-unused-function"]
    objs, todo = [], []
    for src in sources:
        obj = BUILD / f"{src.stem}.host.o"
        objs.append(obj)
        if force or not obj.exists() or obj.stat().st_mtime < src.stat().st_mtime:
            todo.append((src, obj))
    for src, obj in todo:
        cmd = [cxx, *flags, "-c", str(src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), flush=True)
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"compile failed: {src}\n{res.stderr}")
    out = PKG / "_dlgm_host.so"
    if force or todo or not out.exists():
        cmd = [cxx, "-shared", "-fopenmp", *map(str, objs), "-o", str(out), "-lpthread", "-lz"]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed: _dlgm_host.so\n{res.stderr}")
    return out


def build(jobs: int | None = None, verbose: bool = False, force: bool = False) -> list[Path]:
    jobs = jobs or min(8, os.cpu_count() or 4)
    tlib, tinc, abi = _torch_paths()
    common = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", f"-I{CSRC / 'include'}",
              "-Wno-unused-result", "-Wno-deprecated-declarations"]
    torch_flags = [*common, *(f"-I{p}" for p in tinc), f"-I{sysconfig.get_paths()['include']}",
                   f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1", "-DTORCH_API_INCLUDE_EXTENSION_H"]
    kern_src = sorted((CSRC / "kernels").glob("*.hip")) + [CSRC / "bindings.cpp"]
    kern_ld = [f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip", "-ltorch", "-lhipblaslt",
               f"-Wl,-rpath,{tlib}"]
    outs = [_build_lib("_dlgm_hip.so", kern_src, torch_flags, kern_ld, jobs, verbose, force)]
    host_src = sorted((CSRC / "host").glob("*.cpp"))
    if host_src:
        outs.append(_build_host(host_src, jobs, verbose, force))
    return outs


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-f", "--force", action="store_true")
    a = ap.parse_args()
    for p in build(a.jobs, a.verbose, a.force):
        print(p)
    return 0


if __name__ == "__main__":
    sys.exit(main())
