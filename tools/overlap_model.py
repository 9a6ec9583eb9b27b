#!/usr/bin/env python3
"""ZeRO-3 communication overlap with MODELLED xGMI time, at the reference's knobs.

Rank 0 of an 8-rank job alone on one MI355X (tools/shadow_rank.py: true-size shards, gathers and reduce-scatters),
with ShadowComm's link model: every collective holds its communicator's HIP stream for its ring time at a bus
bandwidth of 150 GB/s (one xGMI link) or 350 GB/s, before its local stand-in copy. The consumer waits on the
collective's event exactly as with RCCL, so exposed communication shows up as step time. Configurations:

* Llama-3-8B, the reference's ZeRO-3 knobs (stage3_max_live_parameters = stage3_prefetch_bucket_size-scale 1e9,
  stage3_max_reuse_distance 1e9: ``/root/reference/ai_engine/deepspeed_launcher.py:70-75, 186-194``), per-micro-batch
  gradient reduce-scatter (DeepSpeed's pattern) -- per-layer gathers in the forward AND the backward of every
  micro-batch;
* the same with this engine's local fp32 gradient accumulation (one reduce-scatter per step);
* Llama-3-8B with "hbm" residency (the multi-GPU default: one gather per unit per step);
* Llama-3-70B config 4 (activation checkpointing, the 70b preset's ZeRO-3), "hbm" knobs: 1.71 GB/layer gathers.

Each runs at 0 (no link time), 150 and 350 GB/s; the step time against the zero-delay run is the exposed fraction.
A MODEL, not a measurement of an 8-GPU node: it leaves out the CUs RCCL's channels take and link contention between
concurrent collectives.

    python tools/overlap_model.py --out profiles/zero3_overlap_model_r06.json
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CONFIGS = {
    "llama3-8b_reference_knobs_rs_per_micro": dict(model="llama3-8b", ga=8, live="1e9", reuse="1e9", local="off"),
    "llama3-8b_reference_knobs_local_grads": dict(model="llama3-8b", ga=8, live="1e9", reuse="1e9", local="on"),
    "llama3-8b_hbm": dict(model="llama3-8b", ga=8, live="hbm", reuse="hbm", local="hbm"),
    "llama3-70b_config4_ckpt": dict(model="llama3-70b", ga=2, live="hbm", reuse="hbm", local="hbm", ckpt=True),
}


def run_one(name: str, c: dict, gbps: float, steps: int, warmup: int, outdir: str) -> dict:
    out = os.path.join(outdir, f"{name}_{int(gbps)}.json")
    cmd = [sys.executable, "-u", os.path.join(ROOT, "tools", "shadow_rank.py"), "--model", c["model"], "--world", "8",
           "--rank", "0", "--ga", str(c["ga"]), "--steps", str(steps), "--warmup", str(warmup), "--async-comm",
           "--live-params", c["live"], "--reuse-distance", c["reuse"], "--local-grads", c["local"], "--out", out]
    if c.get("ckpt"):
        cmd.append("--ckpt")
    if gbps > 0:
        cmd += ["--link-gbps", str(gbps)]
    t0 = time.time()
    res = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=900)
    if res.returncode != 0:
        return {"error": res.stderr[-3000:], "rc": res.returncode}
    with open(out) as f:
        rec = json.load(f)
    rec["wall_s"] = round(time.time() - t0, 1)
    return rec


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--configs", default=",".join(CONFIGS))
    ap.add_argument("--gbps", default="0,150,350")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--tmp", default=os.path.join(ROOT, "gpurun_out", "overlap_model"))
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    os.makedirs(a.tmp, exist_ok=True)
    report = {"what": __doc__.split("\n\n")[0], "model_not_measurement": True, "world": 8, "rank": 0, "runs": {}}
    for name in a.configs.split(","):
        c = CONFIGS[name]
        rows = {}
        for g in (float(x) for x in a.gbps.split(",")):
            rec = run_one(name, c, g, a.steps, a.warmup, a.tmp)
            if "error" in rec:
                rows[str(int(g))] = rec
                print(f"[overlap] {name} @ {g:g} GB/s: FAILED rc={rec['rc']}", flush=True)
                break
            timed = rec["step_s"][a.warmup:] or rec["step_s"]
            step = sorted(timed)[len(timed) // 2]
            lm = rec.get("link_model") or {}
            rows[str(int(g))] = {"step_s_median": step, "step_s": rec["step_s"],
                                 "modelled_link_s_per_step": round(lm.get("modelled_link_s_total", 0.0) /
                                                                   max(1, lm.get("steps_in_run", 1)), 3),
                                 "collectives_issued": rec.get("async_collectives_issued"),
                                 "gathers_per_step": rec["knobs"]["gathers_per_step"],
                                 "local_grads": rec["knobs"]["local_grads"], "peak_GiB": rec["peak_GiB"]}
            print(f"[overlap] {name} @ {g:g} GB/s: step {step:.3f}s, link time queued "
                  f"{rows[str(int(g))]['modelled_link_s_per_step']:.3f}s/step", flush=True)
        base = rows.get("0", {}).get("step_s_median")
        for k, r in rows.items():
            if base and "step_s_median" in r:
                r["vs_zero_delay"] = round(r["step_s_median"] / base, 4)
                r["modelled_efficiency_8gpu"] = round(base / r["step_s_median"], 4)
        report["runs"][name] = {"config": c, "by_link_gbps": rows}
    text = json.dumps(report, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)
    print(text[-3000:])
    return 0


if __name__ == "__main__":
    sys.exit(main())
