"""Offline consolidation of a sharded checkpoint into full fp32 (or bf16) weights -- no GPU, no process group.

DeepSpeed ships ``zero_to_fp32.py`` inside every checkpoint directory for this job (SURVEY.md §5.4:
"plus ``zero_to_fp32.py`` recovery"); this is the equivalent for the layout written by
:class:`ckpt.checkpoint.AsyncCheckpointer`::

    <save_dir>/<tag>/mp_rank_00_model_states.pt                               meta (weights_only)
    <save_dir>/<tag>/zero_pp_rank_{r}_mp_rank_00_optim_states.master.bin       rank r's fp32 shards

Each flat group (one transformer block, the embedding, the head) is partitioned in P equal
shards; rank r's file holds its shard of every group at the group's ``shard_off``. The full group
is the concatenation of the P shards, and each parameter sits at its recorded offset inside it.
The shard files are memory-mapped, so consolidating a 70B checkpoint needs host memory for one
group at a time plus the output.

    python -m distributed_llm_training_gpu_manager_amd.ckpt.zero_to_fp32 <save_dir> out.safetensors \\
        [--tag global_step120] [--dtype bf16]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
from typing import Dict, Optional

import numpy as np
import torch

from .checkpoint import STATE, _optim_prefix, complete_tags


def _resolve_tag(save_dir: str, tag: Optional[str]) -> str:
    if tag:
        return tag
    latest = os.path.join(save_dir, "latest")
    if os.path.exists(latest):
        with open(latest) as f:
            return f.read().strip()
    tags = complete_tags(save_dir)
    if not tags:
        raise FileNotFoundError(f"no complete checkpoint under {save_dir}")
    return tags[-1]


def consolidate(save_dir: str, tag: Optional[str] = None, state: str = "master",
                dtype: torch.dtype = torch.float32) -> Dict[str, torch.Tensor]:
    """Full parameters (or an optimizer moment, ``state`` = exp_avg / exp_avg_sq) of one checkpoint."""
    assert state in STATE, state
    d = os.path.join(save_dir, _resolve_tag(save_dir, tag))
    meta = torch.load(os.path.join(d, "mp_rank_00_model_states.pt"), weights_only=True)
    ep = int(meta.get("engine_config", {}).get("expert_parallel_size", 1) or 1)
    if ep > 1:
        raise NotImplementedError("expert-parallel checkpoints hold different experts per EP rank; "
                                  "consolidate them through ZeroEngine.full_params() under the same EP size")
    P = int(meta["partition_count"])
    maps = [np.memmap(os.path.join(d, f"{_optim_prefix(r)}.{state}.bin"), dtype=np.float32, mode="r")
            for r in range(P)]
    out: Dict[str, torch.Tensor] = {}
    for g in meta["groups"]:
        full = np.concatenate([m[g["shard_off"]:g["shard_off"] + g["shard_numel"]] for m in maps])
        for name, off, shape in g["params"]:
            n = math.prod(shape)
            out[f"{g['name']}.{name}"] = torch.from_numpy(np.array(full[off:off + n])).view(*shape).to(dtype)
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("save_dir")
    ap.add_argument("output", help=".safetensors file")
    ap.add_argument("--tag", default=None, help="checkpoint tag (default: 'latest', else the newest complete)")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--state", default="master", choices=list(STATE))
    a = ap.parse_args(argv)
    from safetensors.torch import save_file

    params = consolidate(a.save_dir, a.tag, a.state, torch.float32 if a.dtype == "fp32" else torch.bfloat16)
    save_file({k: v.contiguous() for k, v in params.items()}, a.output)
    n = sum(v.numel() for v in params.values())
    print(json.dumps({"output": a.output, "tensors": len(params), "params": n, "dtype": a.dtype}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
