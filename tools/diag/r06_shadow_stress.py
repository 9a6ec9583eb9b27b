#!/usr/bin/env python3
"""Round 6: how often does the asynchronous shadow run differ from the synchronous one (tests/test_shadow_async_gpu.py
cases), in one process, N repetitions per case. One synchronous reference per case (it repeats bit-exactly: checked
twice). Prints one JSON line per case and a summary."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
import torch  # noqa: E402
import test_shadow_async_gpu as T  # noqa: E402


def history():
    """HISTORY=1: first run the GPU test files the suite runs before tests/test_shadow_async_gpu.py, in this process
    (the mismatches so far appeared only after them), and list the threads they left running."""
    import threading
    import pytest
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
    files = sorted(f for f in os.listdir(os.path.join(root, "tests")) if f.startswith("test_") and f.endswith(".py")
                   and f < "test_shadow_async_gpu.py")
    rc = pytest.main(["-q", "-x", "-m", "gpu", "-p", "no:cacheprovider", "--timeout", "300",
                      "--timeout-method", "thread", *[os.path.join(root, "tests", f) for f in files]])
    th = [(t.name, t.daemon, t.is_alive()) for t in threading.enumerate()]
    print(json.dumps({"history_rc": int(rc), "threads_after_history": th}), flush=True)


def main():
    if os.environ.get("HISTORY") == "1":
        history()
    reps = int(os.environ.get("REPS", "20"))
    cases = os.environ.get("CASES", "zero3_nonresident,zero3_offload_param,zero3_nonresident_local,zero2").split(",")
    out = {"env": {k: os.environ.get(k) for k in ("HSA_ENABLE_SDMA", "DLGM_SHADOW_DELAY", "GPU_MAX_HW_QUEUES")},
           "reps": reps, "cases": {}}
    for case in cases:
        kw = T.CASES[case]
        ref, _ = T._run("llama-tiny", 4, False, **kw)
        ref2, _ = T._run("llama-tiny", 4, False, **kw)
        same = lambda a, b: all(torch.equal(a[k], b[k]) for k in T.STATE)  # noqa: E731
        bad, t0, where = 0, time.time(), []
        for i in range(reps):
            got, _ = T._run("llama-tiny", 4, True, **kw)
            if not same(ref, got):
                bad += 1
                k0 = next(k for k in T.STATE if not torch.equal(ref[k], got[k]))
                where.append((i, k0, T._where(ref, got, k0)["max_abs"]))
        rec = {"ref_repeats": same(ref, ref2), "async_mismatches": bad, "of": reps, "first": where[:5],
               "s": round(time.time() - t0, 1)}
        out["cases"][case] = rec
        print(json.dumps({case: rec}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
