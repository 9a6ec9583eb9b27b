"""RCCL collective microbenchmark over xGMI (rccl-tests style): bus bandwidth vs message size.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/comm_bench.py \
        --ops all_gather,reduce_scatter,all_reduce,all_to_all --min-mb 1 --max-mb 1024

Bus bandwidth uses the rccl-tests conventions: algbw = bytes / time; busbw = algbw * factor with
factor (W-1)/W for all_gather / reduce_scatter / all_to_all and 2(W-1)/W for all_reduce. On an
8x MI355X node (7 xGMI links per GPU, ~153 GB/s each) a single ring is bound by one link; the
engine's bucket policy (one transformer block per collective) sits at the
right end of this curve. Runs on gloo/CPU too (tests use it as a smoke check).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from distributed_llm_training_gpu_manager_amd.parallel.comm import Comm, init_distributed  # noqa: E402
from distributed_llm_training_gpu_manager_amd.utils.commbench import FACTOR, run  # noqa: E402


def main(argv=None) -> list:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="all_gather,reduce_scatter,all_reduce,all_to_all")
    ap.add_argument("--min-mb", type=float, default=1.0)
    ap.add_argument("--max-mb", type=float, default=1024.0)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    env = init_distributed()
    comm = Comm()
    dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    rows = []
    for op in a.ops.split(","):
        mb = a.min_mb
        while mb <= a.max_mb + 1e-9:
            nbytes = int(mb * (1 << 20))
            dt = run(op, comm, nbytes, env.device, dtype, a.iters, a.warmup)
            algbw = nbytes / dt / 1e9
            rec = {"op": op, "bytes": nbytes, "time_us": dt * 1e6, "algbw_GBps": algbw,
                   "busbw_GBps": algbw * FACTOR[op](comm.world), "world": comm.world, "backend": env.backend}
            rows.append(rec)
            if env.rank == 0:
                print(json.dumps(rec), flush=True)
            mb *= 2
    if env.rank == 0 and a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)
    return rows


if __name__ == "__main__":
    main()
