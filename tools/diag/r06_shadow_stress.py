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
    import contextlib
    from distributed_llm_training_gpu_manager_amd.utils import stream_audit as sa
    with contextlib.ExitStack() as st:
        if os.environ.get("POISON") == "1":  # uninitialised float allocations read as NaN
            st.enter_context(sa.poison_allocations())
        audit = st.enter_context(sa.stream_audit()) if os.environ.get("AUDIT") == "1" else None
        body()
    if audit is not None:
        print(json.dumps({"audit": audit.report()[:4000]}), flush=True)


def patch_variant(v):
    """Diagnostic variants of ShadowComm._run (run under AMD_SERIALIZE_KERNEL/COPY=3, where no stream ordering is
    needed): 'norecord' skips record_stream of the collective's tensors; 'samestream' runs the stand-in on the
    issuing stream (no comm-stream allocations) but keeps the asynchronous handle."""
    from distributed_llm_training_gpu_manager_amd.parallel import comm as C
    orig = C.ShadowComm._run

    def run(self, fn, tensors, async_op, link_ns=0):
        if not self.async_mode or not tensors or not tensors[0].is_cuda:
            return orig(self, fn, tensors, async_op, link_ns)
        dev = tensors[0].device
        cur = torch.cuda.current_stream(dev)
        if v == "samestream":
            if self.delay_cycles:
                torch.cuda._sleep(self.delay_cycles)
            fn()
            ev = torch.cuda.Event()
            ev.record(cur)
        else:
            if self._stream is None:
                from distributed_llm_training_gpu_manager_amd.utils.streams import owned_stream
                self._stream = owned_stream(dev, "shadow-comm")
            s = self._stream
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                if self.delay_cycles:
                    torch.cuda._sleep(self.delay_cycles)
                fn()
                ev = torch.cuda.Event()
                ev.record(s)
        self.issued += 1
        h = C.Handle(post=lambda: torch.cuda.current_stream(dev).wait_event(ev))
        if not async_op:
            h.wait()
        return h
    C.ShadowComm._run = run


def patch_mesh():
    """MESH_ALLOC=<uncached|fine-grained|coarse-grained>: the heap's memory kind; MESH_KEEP=1: never free a heap (every
    mesh's heap tensor is kept referenced for the life of the process)."""
    from distributed_llm_training_gpu_manager_amd.parallel import xgmi_mesh as X
    orig = X.XgmiMesh.__init__
    keep = []

    def init(self, comm, device, regions, timeout_s=60.0, alloc_mode="auto"):
        orig(self, comm, device, regions, timeout_s, os.environ.get("MESH_ALLOC", alloc_mode))
        if os.environ.get("MESH_KEEP") == "1":
            keep.append(self.heap)
    X.XgmiMesh.__init__ = init


def body():
    import gc
    patch_mesh()
    if os.environ.get("VARIANT"):
        patch_variant(os.environ["VARIANT"])
    if os.environ.get("NOGC") == "1":  # no cyclic collection at all: dead engines' tensors are never freed mid-run
        gc.disable()
    if os.environ.get("GCEACH") == "1":  # collect before every run: nothing of an older engine is freed during one
        orig = T._run

        def run_collected(*a, **k):
            gc.collect()
            torch.cuda.synchronize()
            return orig(*a, **k)
        T._run = run_collected
    if os.environ.get("HISTORY") == "1":
        history()
    reps = int(os.environ.get("REPS", "20"))
    cases = os.environ.get("CASES", ",".join(sorted(T.CASES))).split(",")
    out = {"env": {k: os.environ.get(k) for k in ("HSA_ENABLE_SDMA", "DLGM_SHADOW_DELAY", "GPU_MAX_HW_QUEUES")},
           "reps": reps, "cases": {}}
    same = lambda a, b: all(torch.equal(a[k], b[k]) for k in T.STATE)  # noqa: E731
    refs = {}
    for case in cases:  # synchronous references (each checked to repeat)
        ref, _ = T._run("llama-tiny", 4, False, **T.CASES[case])
        ref2, _ = T._run("llama-tiny", 4, False, **T.CASES[case])
        refs[case] = ref
        out["cases"][case] = {"ref_repeats": same(ref, ref2), "async_mismatches": 0, "of": 0, "first": []}
    t0 = time.time()
    mode = os.environ.get("LOOP_MODE", "async")  # async | sync: the interleaved runs asynchronous or synchronous
    for i in range(reps):  # the cases interleaved, as consecutive tests run them (mesh cases between the others)
        for case in cases:
            got, _ = T._run("llama-tiny", 4, mode == "async", **T.CASES[case])
            rec = out["cases"][case]
            rec["of"] += 1
            if not same(refs[case], got):
                rec["async_mismatches"] += 1
                k0 = next(k for k in T.STATE if not torch.equal(refs[case][k], got[k]))
                if len(rec["first"]) < 5:
                    rec["first"].append((i, k0, T._where(refs[case], got, k0)["max_abs"]))
    out["s"] = round(time.time() - t0, 1)
    for case in cases:
        print(json.dumps({case: out["cases"][case]}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
