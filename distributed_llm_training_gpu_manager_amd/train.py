"""Entry point run by the launcher on every rank: ``python -m distributed_llm_training_gpu_manager_amd.train``.

Restart warm-up: device memory another process has just freed costs a new process ~20 ms per
GiB to allocate (the driver reclaims it; a second allocation of memory this process freed itself is free --
tools/diag/r05/vram_alloc.py: 3.2 s for 160 GiB after a predecessor, 0.0 s within one process). A relaunched rank
would pay that inside its engine construction, after ~2 s of imports. So before importing anything heavy, a
thread allocates and frees, through the HIP runtime directly, the device memory the previous attempt's engine
held (recorded by the trainer as ``<save dir>/.engine_vram_gib.r<rank>``), while this thread imports torch.
"""
import os
import sys
import threading


def _save_dir(argv):
    for i, a in enumerate(argv):
        if a == "--save-dir" and i + 1 < len(argv):
            return argv[i + 1]
        if a.startswith("--save-dir="):
            return a.split("=", 1)[1]
    return os.environ.get("DLGM_SAVE_DIR")


def _prewarm_vram(gib: float, device: int) -> None:
    import ctypes
    try:
        lib = ctypes.CDLL("libamdhip64.so")
        lib.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        lib.hipFree.argtypes = [ctypes.c_void_p]
        if lib.hipSetDevice(device) != 0:
            return
        p = ctypes.c_void_p()
        if lib.hipMalloc(ctypes.byref(p), int(gib * (1 << 30))) == 0:
            lib.hipFree(p)
    except OSError:
        pass


def start_prewarm(argv=None) -> "threading.Thread | None":
    d = _save_dir(sys.argv[1:] if argv is None else argv)
    rank = os.environ.get("RANK", "0")
    if not d or os.environ.get("DLGM_RESTART", "0") == "0":
        return None  # first launch: nothing freed the memory just before
    try:
        with open(os.path.join(d, f".engine_vram_gib.r{rank}")) as f:
            gib = float(f.read().strip())
    except (OSError, ValueError):
        return None
    th = threading.Thread(target=_prewarm_vram, args=(gib, int(os.environ.get("LOCAL_RANK", "0"))), daemon=True,
                          name="vram-prewarm")
    th.start()
    return th


if __name__ == "__main__":
    _th = start_prewarm()
    if _th is not None:  # the trainer joins it before building the engine (never two claims on the HBM at once)
        if __package__ in (None, ""):
            sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import distributed_llm_training_gpu_manager_amd as _pkg
        _pkg._VRAM_PREWARM = _th

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from distributed_llm_training_gpu_manager_amd.engine.trainer import main
else:
    from .engine.trainer import main

if __name__ == "__main__":
    sys.exit(main())
