"""Round 5, 70B rank-scale MTTR: where does the first step after a SIGKILL + shm restore go? Three processes of
tools/probe_startup.py (rank 0 of an 8-rank Llama-3-70B ZeRO-3 job alone on this GPU):
  killed  : 2 steps, save into the /dev/shm tier after step 2, SIGKILL itself (the drill's crash)
  resumed : restore from that snapshot, 3 steps timed unit by unit (buffer preparation after step 1)
  fresh   : 2 steps timed unit by unit, no checkpointer (the baseline first step)
Each child is started as a subprocess (no exec); a SIGKILL of `killed` is the expected outcome."""
import json
import os
import subprocess
import sys
import time

OUT = "gpurun_out/digest"
os.makedirs(OUT, exist_ok=True)
base = [sys.executable, "-u", "tools/probe_startup.py", "--model", os.environ.get("MODEL", "llama3-70b")]
ck = "/tmp/dlgm_resume_probe_ck"
runs = {
    "killed": base + ["--ckpt-tier", "shm", "--steps", "2", "--per-unit", "0", "--save-after", "1", "--save-dir", ck,
                      "--kill-after-save"],
    "resumed": base + ["--ckpt-tier", "shm", "--resume", "--steps", "3", "--per-unit", "1", "--save-dir", ck],
    "fresh": base + ["--steps", "2", "--per-unit", "1"],
}
res = {}
for name in os.environ.get("RUNS", "killed,resumed,fresh").split(","):
    t0 = time.time()
    p = subprocess.run(runs[name] + ["--out", f"{OUT}/resume_{name}.json"], capture_output=True, text=True,
                       timeout=400)
    res[name] = {"rc": p.returncode, "wall_s": round(time.time() - t0, 2), "tail": (p.stdout + p.stderr)[-1500:]}
    print(name, res[name]["rc"], res[name]["wall_s"], flush=True)
    ok = p.returncode == 0 or (name == "killed" and p.returncode == -9)
    if not ok:
        print(res[name]["tail"], flush=True)
        break
for p_ in os.listdir("/dev/shm"):
    if p_.startswith("dlgm-ckpt-"):
        os.unlink(os.path.join("/dev/shm", p_))
with open(f"{OUT}/resume_probe.json", "w") as f:
    json.dump(res, f, indent=1)
sys.exit(0 if all(v["rc"] in (0, -9) for v in res.values()) else 1)
