#!/usr/bin/env python3
"""Post-bench xGMI mesh sweep: the device-driven mesh all-gather / reduce-scatter (parallel/xgmi_mesh.py) beside
RCCL's ring rows at the same sizes, in a process of its own.

bench.py starts one of these per rank as a CHILD process after its result line has been printed and its own process
group destroyed (RANK / WORLD_SIZE / LOCAL_RANK inherited from torchrun, a fresh MASTER_PORT agreed beforehand), so a
new transport can never cost the headline measurement. Rank 0 prints one ``[mesh-sweep] {...}`` line (bench.py
routes it to stderr) and, when ``DLGM_SWEEP_DIR`` names a directory, writes ``mesh_sweep_w{W}.json`` there.
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main() -> int:
    import torch
    import torch.distributed as dist

    from distributed_llm_training_gpu_manager_amd.parallel.comm import Comm, init_distributed
    from distributed_llm_training_gpu_manager_amd.utils.commbench import MESH_OPS, sweep

    env = init_distributed("cuda" if torch.cuda.is_available() else "cpu")
    comm = Comm()
    rows = []
    if env.device.type == "cuda" and env.world > 1:
        rows = sweep(comm, env.device, ops=MESH_OPS + ("all_gather", "reduce_scatter", "all_to_all"),
                     sizes_mb=(16, 64, 256))
    if env.rank == 0:
        rec = {"mesh_sweep": rows, "world": env.world}
        print("[mesh-sweep] " + json.dumps(rec), flush=True)
        d = os.environ.get("DLGM_SWEEP_DIR")
        if d and os.path.isdir(d):
            with open(os.path.join(d, f"mesh_sweep_w{env.world}.json"), "w") as f:
                json.dump(rec, f, indent=1)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
