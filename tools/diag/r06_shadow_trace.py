#!/usr/bin/env python3
"""Round 6: find the first op whose result differs between the synchronous and an asynchronous shadow run of TARGET.

Every op's written tensors (outputs, Tensor(a!) arguments) are checksummed right after it runs (device synchronised
first: AMD_SERIALIZE_KERNEL=3 showed the same mismatch pattern, so execution order is not what differs). The case
sequence of tools/diag/r06_shadow_stress.py (references of every case, then every case asynchronously, REPS times)
reproduces the mismatch; the target's synchronous trace is compared with each asynchronous one."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402
import test_shadow_async_gpu as T  # noqa: E402


STRUCT = os.environ.get("STRUCT", "0") == "1"


class Trace(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.ops = []

    @staticmethod
    def _sums(ts):
        sums = []
        for t in ts:
            x = t.detach()
            if x.is_floating_point():
                x = x.double()
                sums.append((float(x.nan_to_num(123.0).sum()), float(x.abs().nan_to_num(123.0).sum()),
                             bool(torch.isfinite(x).all())))
            else:
                sums.append((int(x.long().sum()),))
        return sums

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        name = str(func.name()) if hasattr(func, "name") else str(func)
        if STRUCT:  # op, shapes, strides, dtypes, current stream kind: no device work, no allocation
            out = func(*args, **kwargs)
            flat = [a for a in list(args) + list(kwargs.values()) if isinstance(a, torch.Tensor)]
            self.ops.append((name, [(tuple(t.shape), tuple(t.stride()), str(t.dtype)[6:]) for t in flat], [], [],
                             len(self.ops)))
            return out
        skip = name.startswith("c10d::") or "record_stream" in name or name in ("aten::empty", "aten::empty_strided")
        ins = []
        if not skip:
            flat = []
            for a in list(args) + list(kwargs.values()):
                if isinstance(a, torch.Tensor):
                    flat.append(a)
                elif isinstance(a, (list, tuple)):
                    flat += [v for v in a if isinstance(v, torch.Tensor)]
            flat = [t for t in flat if t.is_cuda and t.numel() > 0]
            if flat:
                torch.cuda.synchronize()
                ins = self._sums(flat)
        out = func(*args, **kwargs)
        if skip:
            return out
        try:
            sch = func._schema
            wr = [a for i, a in enumerate(args) if i < len(sch.arguments) and sch.arguments[i].alias_info is not None
                  and sch.arguments[i].alias_info.is_write]
            wr += [v for k, v in kwargs.items() for sa in sch.arguments if sa.name == k and sa.alias_info is not None
                   and sa.alias_info.is_write]
        except Exception:
            wr = []
        ts = [t for t in ([out] if isinstance(out, torch.Tensor) else list(out) if isinstance(out, (tuple, list)) else [])
              if isinstance(t, torch.Tensor)] + [t for t in wr if isinstance(t, torch.Tensor)]
        ts = [t for t in ts if t.is_cuda and t.numel() > 0]
        if ts or ins:
            torch.cuda.synchronize()
            self.ops.append((name, [tuple(t.shape) for t in ts], self._sums(ts), ins, len(self.ops)))
        return out


def run(case, async_mode, trace):
    if trace is None:
        return T._run("llama-tiny", 4, async_mode, **T.CASES[case])[0], None
    tr = Trace()
    with tr:
        r, _ = T._run("llama-tiny", 4, async_mode, **T.CASES[case])
    return r, tr.ops


def first_diff(a, b):
    # the async trace has extra ops? align by index of (name, shapes)
    i = j = 0
    while i < len(a) and j < len(b):
        if a[i][0] != b[j][0] or a[i][1] != b[j][1]:
            return {"structure_diverges_at": i, "sync": a[i][:2], "async": b[j][:2],
                    "sync_prev": [x[:2] for x in a[max(0, i - 4):i]], "async_prev": [x[:2] for x in b[max(0, j - 4):j]]}
        if a[i][3] != b[j][3]:  # inputs differ while every earlier output matched: written behind the ops' backs
            return {"first_INPUT_diff_at": i, "op": a[i][0], "shapes": a[i][1], "sync_in": a[i][3],
                    "async_in": b[j][3], "prev": [(x[0], x[1]) for x in a[max(0, i - 8):i]], "n_ops": (len(a), len(b))}
        if a[i][2] != b[j][2]:
            return {"first_value_diff_at": i, "op": a[i][0], "shapes": a[i][1], "sync": a[i][2], "async": b[j][2],
                    "sync_in": a[i][3], "async_in": b[j][3],
                    "prev": [(x[0], x[1]) for x in a[max(0, i - 8):i]], "n_ops": (len(a), len(b))}
        i += 1
        j += 1
    return {"no_diff_in_common_prefix": (len(a), len(b))}


def main():
    target = os.environ.get("TARGET", "zero2")
    reps = int(os.environ.get("REPS", "6"))
    cases = sorted(T.CASES)
    same = lambda x, y: all(torch.equal(x[k], y[k]) for k in T.STATE)  # noqa: E731
    refs = {c: run(c, False, None)[0] for c in cases}
    ref_t, sync_ops = run(target, False, True)
    print(json.dumps({"traced_sync_equals_ref": same(ref_t, refs[target]), "sync_ops": len(sync_ops)}), flush=True)
    found = 0
    for i in range(reps):
        for c in cases:
            if c != target:
                run(c, True, None)
                continue
            got, ops = run(c, True, True)
            ok = same(refs[target], got)
            rec = {"rep": i, "equal": ok}
            if not ok:
                found += 1
                rec["diff"] = first_diff(sync_ops, ops)
            print(json.dumps(rec, default=str), flush=True)
            if found >= 2:
                return


if __name__ == "__main__":
    main()
