#!/usr/bin/env python3
"""Communication / compute overlap from a rocprofv3 kernel trace of a shadow-rank run with the link model
(tools/overlap_model.py, ShadowComm link_gbps): the modelled link time is the `spin_kernel` dispatches on the
communicators' streams; compute is every kernel on the stream that runs the model's fwd / bwd (the busiest one).

    rocprofv3 --kernel-trace --output-format csv -d out -o run -- python tools/shadow_rank.py ... --link-gbps 350
    python tools/trace_overlap.py out/run_kernel_trace.csv [--out summary.json]

Reported: total spin time, the part of it during which the compute stream was running a kernel (hidden), the
compute stream's idle time inside the traced window, the idle gaps that coincide with a spin (exposed link time),
and the largest such gaps with the compute kernels around them.
"""
from __future__ import annotations

import argparse
import csv
import json
import sys
from collections import defaultdict
from typing import Dict, List, Tuple


def _merge(iv: List[Tuple[int, int]]) -> List[Tuple[int, int]]:
    out: List[Tuple[int, int]] = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], b))
        else:
            out.append((a, b))
    return out


def _overlap(a: List[Tuple[int, int]], b: List[Tuple[int, int]]) -> int:
    i = j = tot = 0
    while i < len(a) and j < len(b):
        lo, hi = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if lo < hi:
            tot += hi - lo
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def analyse(path: str, skip_s: float = 0.0) -> Dict:
    rows = list(csv.DictReader(open(path)))
    by_stream: Dict[str, List[Tuple[int, int, str]]] = defaultdict(list)
    for r in rows:
        by_stream[r["Stream_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    spins = [(a, b) for ks in by_stream.values() for a, b, n in ks if "spin_kernel" in n]
    compute_sid = max(by_stream, key=lambda s: sum(b - a for a, b, n in by_stream[s] if "spin_kernel" not in n))
    comp = sorted(by_stream[compute_sid])
    t0 = comp[0][0] + int(skip_s * 1e9)
    comp = [k for k in comp if k[0] >= t0]
    spins = [s for s in spins if s[0] >= t0]
    t1 = comp[-1][1]
    comp_iv = _merge([(a, b) for a, b, _ in comp])
    spin_iv = _merge(spins)
    gaps = [(comp_iv[i][1], comp_iv[i + 1][0]) for i in range(len(comp_iv) - 1)]
    exposed = _overlap(gaps, spin_iv)
    spin_total = sum(b - a for a, b in spin_iv)
    busy = sum(b - a for a, b in comp_iv)
    big = sorted(((b - a, a, b) for a, b in gaps), reverse=True)[:8]
    names = {(a, b): n for a, b, n in comp}
    ends = sorted((b, n) for a, b, n in comp)

    def before(t):
        import bisect
        k = bisect.bisect_right([e for e, _ in ends], t) - 1
        return ends[k][1][:60] if k >= 0 else None
    return {"trace": path, "window_s": round((t1 - t0) / 1e9, 3), "compute_stream": compute_sid,
            "compute_busy_s": round(busy / 1e9, 3), "compute_idle_s": round((t1 - t0 - busy) / 1e9, 3),
            "link_spin_s": round(spin_total / 1e9, 3),
            "link_hidden_s": round(_overlap(comp_iv, spin_iv) / 1e9, 3),
            "link_exposed_s": round(exposed / 1e9, 3),
            "hidden_fraction": round(1 - exposed / spin_total, 4) if spin_total else None,
            "largest_idle_gaps": [{"ms": round(d / 1e6, 3), "after": before(a),
                                   "during_spin_ms": round(_overlap([(a, b)], spin_iv) / 1e6, 3)} for d, a, b in big],
            "streams": {s: {"kernels": len(k), "busy_s": round(sum(b - a for a, b, _ in k) / 1e9, 3),
                            "spins": sum(1 for *_, n in k if "spin_kernel" in n)} for s, k in by_stream.items()}}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("trace")
    ap.add_argument("--skip-s", type=float, default=0.0, help="ignore the first seconds of the trace (init, warmup)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rep = analyse(a.trace, a.skip_s)
    text = json.dumps(rep, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)
    print(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
