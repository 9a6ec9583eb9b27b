#!/usr/bin/env python3
"""Post-bench transport checks and xGMI mesh sweep, in a process of its own.

bench.py starts one of these per rank as a CHILD process after its result line has been printed and its own process
group destroyed (RANK / WORLD_SIZE / LOCAL_RANK inherited from torchrun, a fresh MASTER_PORT agreed beforehand), so a
new transport can never cost the headline measurement. First it CHECKS, on the same inputs across the real devices,
that the mesh all-gather / reduce-scatter / EP dispatch-combine are bit-exact against RCCL and that two llama-tiny
ZeRO-3 steps on RCCL and on the mesh match one process (utils/meshcheck.py): rank 0 prints one
``[mesh-check] {...}`` line. Then, on the GPU, it measures the device-driven mesh all-gather / reduce-scatter /
all-to-all beside RCCL's rows at the same sizes: one ``[mesh-sweep] {...}`` line. bench.py routes this process's
output to stderr; with ``DLGM_SWEEP_DIR`` both records are also written there (``mesh_check_w{W}.json``,
``mesh_sweep_w{W}.json``).
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

    from distributed_llm_training_gpu_manager_amd.utils.meshcheck import run_checks

    env = init_distributed("cuda" if torch.cuda.is_available() else "cpu")
    comm = Comm()
    d = os.environ.get("DLGM_SWEEP_DIR")
    if env.world > 1 and os.environ.get("DLGM_MESH_CHECK", "1") != "0":
        chk = run_checks(comm, env.device)
        if env.rank == 0:
            print("[mesh-check] " + json.dumps(chk), file=sys.stderr, flush=True)
            if d and os.path.isdir(d):
                with open(os.path.join(d, f"mesh_check_w{env.world}.json"), "w") as f:
                    json.dump(chk, f, indent=1)
    rows = []
    if env.device.type == "cuda" and env.world > 1 and os.environ.get("DLGM_MESH_SWEEP", "1") != "0":
        rows = sweep(comm, env.device, ops=MESH_OPS + ("all_gather", "reduce_scatter", "all_to_all"),
                     sizes_mb=(16, 64, 256))
    if env.rank == 0 and rows:
        rec = {"mesh_sweep": rows, "world": env.world}
        print("[mesh-sweep] " + json.dumps(rec), file=sys.stderr, flush=True)
        if d and os.path.isdir(d):
            with open(os.path.join(d, f"mesh_sweep_w{env.world}.json"), "w") as f:
                json.dump(rec, f, indent=1)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
