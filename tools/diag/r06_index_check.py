#!/usr/bin/env python3
"""Round 6: bounds-check every indexing op of the interleaved shadow sequence on the GPU (indices read to the host
BEFORE the op runs; a violation is reported with its stack instead of being executed), to test whether an
out-of-range gather explains the history-dependent asynchronous mismatch (and the hardware exception a
vectorized_gather_kernel raised once the allocator's free blocks had been released with empty_cache)."""
import json
import os
import sys
import traceback

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402
import test_shadow_async_gpu as T  # noqa: E402

aten = torch.ops.aten
VIOL = []
SEEN = {}


class Bounds(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        name = str(func.name()) if hasattr(func, "name") else str(func)
        chk = None
        try:
            if name in ("aten::index_select", "aten::embedding"):
                if name == "aten::index_select":
                    src, dim, idx = args[0], args[1], args[2]
                else:
                    src, idx, dim = args[0], args[1], 0
                chk = (src.shape[dim], idx)
            elif name in ("aten::gather", "aten::scatter_add_", "aten::scatter_", "aten::scatter_add", "aten::scatter"):
                src, dim, idx = args[0], args[1], args[2]
                chk = (src.shape[dim], idx)
            elif name in ("aten::index.Tensor", "aten::index_put_", "aten::index_put", "aten::_index_put_impl_"):
                src, ind = args[0], args[1]
                for d, ix in enumerate(ind):
                    if ix is not None and ix.dtype in (torch.int64, torch.int32):
                        self._one(name, src.shape[d], ix)
            if chk is not None and chk[1].numel() and chk[1].dtype in (torch.int64, torch.int32):
                self._one(name, chk[0], chk[1])
        except _Bad:
            raise
        except Exception as e:  # noqa: BLE001
            VIOL.append({"op": name, "check_error": repr(e)})
        key = name
        SEEN[key] = SEEN.get(key, 0) + 1
        return func(*args, **kwargs)

    @staticmethod
    def _one(name, size, idx):
        lo, hi = int(idx.min()), int(idx.max())
        if lo < -size or hi >= size:
            VIOL.append({"op": name, "size": int(size), "min": lo, "max": hi, "n": int(idx.numel()),
                         "stack": "".join(traceback.format_stack(limit=12)[:-2])[-2500:]})
            raise _Bad(f"{name}: index range [{lo}, {hi}] for size {size}")


class _Bad(RuntimeError):
    pass


def main():
    reps = int(os.environ.get("REPS", "3"))
    cases = sorted(T.CASES)
    out = {"cases": {}}
    with Bounds():
        for c in cases:
            try:
                T._run("llama-tiny", 4, False, **T.CASES[c])
            except _Bad as e:
                out["cases"][c + ":sync"] = str(e)
        for i in range(reps):
            for c in cases:
                try:
                    T._run("llama-tiny", 4, True, **T.CASES[c])
                except _Bad as e:
                    out["cases"][f"{c}:async{i}"] = str(e)
    out["violations"] = VIOL[:6]
    out["n_violations"] = len(VIOL)
    out["index_ops_seen"] = {k: v for k, v in SEEN.items() if "index" in k or "gather" in k or "embedding" in k
                             or "scatter" in k}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
