#!/usr/bin/env python3
"""Round 6: which preceding engine makes the next asynchronous shadow run differ? For each case X, REPS times: run X
(async), then the target case (async), and compare the target with its synchronous reference. Then the details of one
mismatch: per state tensor, the differing elements by parameter and the largest gradient differences."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
import torch  # noqa: E402
import test_shadow_async_gpu as T  # noqa: E402


def detail(ref, got, eng_layout):
    out = {}
    for k in T.STATE:
        d = (ref[k].float() - got[k].float()).abs()
        bad = (d > 0).nonzero().flatten()
        if bad.numel() == 0:
            continue
        top = torch.topk(d, min(8, d.numel())).indices.tolist()
        where = []
        for i in top:
            for gi, off, n, names in eng_layout:
                if off <= i < off + n:
                    where.append({"i": i, "group": gi, "off_in_shard": i - off, "ref": float(ref[k][i]),
                                  "got": float(got[k][i])})
        out[k] = {"n_bad": int(bad.numel()), "first_bad": bad[:6].tolist(), "top": where}
    return out


def main():
    reps = int(os.environ.get("REPS", "3"))
    target = os.environ.get("TARGET", "zero3_offload_param")
    same = lambda a, b: all(torch.equal(a[k], b[k]) for k in T.STATE)  # noqa: E731
    ref, _ = T._run("llama-tiny", 4, False, **T.CASES[target])
    res, shown = {}, False
    for x in ["none"] + sorted(T.CASES):
        bad = 0
        for _ in range(reps):
            if x != "none":
                T._run("llama-tiny", 4, True, **T.CASES[x])
            got, _ = T._run("llama-tiny", 4, True, **T.CASES[target])
            if not same(ref, got):
                bad += 1
                if not shown:
                    shown = True
                    print(json.dumps({"after": x, "detail": detail(ref, got, ref["_layout"])}), flush=True)
        res[x] = bad
        print(json.dumps({"after": x, "target": target, "mismatches": bad, "of": reps}), flush=True)
    print(json.dumps({"target": target, "mismatches_after": res}))


if __name__ == "__main__":
    main()
