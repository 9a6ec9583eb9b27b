#!/usr/bin/env python3
"""Compute-stream occupancy from a rocprofv3 kernel trace of a shadow-rank run, for comparing the same configuration
with and without ShadowComm's link model (tools/overlap_model.py): compute is every kernel on the stream that runs the
model's fwd / bwd (the busiest one). Exposed communication shows up as idle time of that stream; a model that slowed
the compute kernels themselves shows up as busy time (the first link model, a spinning one-wave kernel, did: +8.4 %).
Link time modelled by a spinning kernel (`spin_kernel`) is also matched against the idle gaps directly.

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


def analyse(path: str, skip_s: float = 0.0, last_step: bool = False) -> Dict:
    rows = list(csv.DictReader(open(path)))
    by_stream: Dict[str, List[Tuple[int, int, str]]] = defaultdict(list)
    for r in rows:
        by_stream[r["Stream_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    spins = [(a, b) for ks in by_stream.values() for a, b, n in ks if "spin_kernel" in n]
    compute_sid = max(by_stream, key=lambda s: sum(b - a for a, b, n in by_stream[s] if "spin_kernel" not in n))
    comp = sorted(by_stream[compute_sid])
    t0 = comp[0][0] + int(skip_s * 1e9)
    if last_step:  # the window starts where the previous optimizer step ended (its last AdamW kernel)
        ad = [b for ks in by_stream.values() for a, b, n in ks if "adamw" in n.lower()]
        ad.sort()
        if len(ad) >= 2:
            # AdamW launches of one step come in a burst: the previous step's burst is the one before the last gap
            ends = [ad[i] for i in range(len(ad) - 1) if ad[i + 1] - ad[i] > 50_000_000] or [ad[0]]
            t0 = max(t0, ends[-1])
    comp = [k for k in comp if k[0] >= t0]
    spins = [s for s in spins if s[0] >= t0]
    t1 = comp[-1][1]
    comp_iv = _merge([(a, b) for a, b, _ in comp])
    spin_iv = _merge(spins)
    gaps = [(comp_iv[i][1], comp_iv[i + 1][0]) for i in range(len(comp_iv) - 1)]
    exposed = _overlap(gaps, spin_iv)
    spin_total = sum(b - a for a, b in spin_iv)
    busy = sum(b - a for a, b in comp_iv)
    gaps = [(a, b) for a, b in gaps if b > a]
    big = sorted(((b - a, a, b) for a, b in gaps), reverse=True)[:10]
    ends = sorted((b, n) for a, b, n in comp)

    import bisect
    end_ts = [e for e, _ in ends]
    starts = sorted((a, n) for a, b, n in comp)
    start_ts = [s_ for s_, _ in starts]

    def before(t):
        k = bisect.bisect_right(end_ts, t) - 1
        return ends[k][1][:70] if k >= 0 else None

    def after(t):
        k = bisect.bisect_left(start_ts, t)
        return starts[k][1][:70] if k < len(starts) else None
    return {"trace": path, "window_s": round((t1 - t0) / 1e9, 3), "compute_stream": compute_sid,
            "compute_busy_s": round(busy / 1e9, 3), "compute_idle_s": round((t1 - t0 - busy) / 1e9, 3),
            "link_spin_s": round(spin_total / 1e9, 3),
            "link_hidden_s": round(_overlap(comp_iv, spin_iv) / 1e9, 3),
            "link_exposed_s": round(exposed / 1e9, 3),
            "hidden_fraction": round(1 - exposed / spin_total, 4) if spin_total else None,
            "idle_gaps_over_1ms": sum(1 for a, b in gaps if b - a > 1_000_000),
            "idle_in_gaps_over_1ms_s": round(sum(b - a for a, b in gaps if b - a > 1_000_000) / 1e9, 3),
            "largest_idle_gaps": [{"ms": round(d / 1e6, 3), "after": before(a), "before": after(b),
                                   "during_spin_ms": round(_overlap([(a, b)], spin_iv) / 1e6, 3)} for d, a, b in big],
            "streams": {s: {"kernels": len(k), "busy_s": round(sum(b - a for a, b, _ in k) / 1e9, 3),
                            "spins": sum(1 for *_, n in k if "spin_kernel" in n)} for s, k in by_stream.items()}}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("trace")
    ap.add_argument("--skip-s", type=float, default=0.0, help="ignore the first seconds of the trace (init, warmup)")
    ap.add_argument("--last-step", action="store_true", help="only the last optimizer step of the trace")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    rep = analyse(a.trace, a.skip_s, a.last_step)
    text = json.dumps(rep, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)
    print(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
