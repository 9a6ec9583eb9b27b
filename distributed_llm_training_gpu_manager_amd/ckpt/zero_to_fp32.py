"""Offline consolidation of a sharded checkpoint into full fp32 (or bf16) weights -- no GPU, no process group.

DeepSpeed ships ``zero_to_fp32.py`` inside every checkpoint directory for this job (SURVEY.md §5.4:
"plus ``zero_to_fp32.py`` recovery"); this is the equivalent for the layout written by
:class:`ckpt.checkpoint.AsyncCheckpointer`::

    <save_dir>/<tag>/mp_rank_00_model_states.pt                      meta (torch.load weights_only)
    <save_dir>/<tag>/zero_pp_rank_{r}_mp_rank_00_optim_states.pt      rank r's fp32 shards (torch.save zip)
    <save_dir>/<tag>/manifest_r{r}.json                               where each record's bytes start

Each flat group (one transformer block, the embedding, the head) is partitioned in P equal shards; the
full group is the concatenation of the P shards and each parameter sits at its recorded offset inside
it. Expert groups (Mixtral, EP > 1) are concatenated over the EP ranks in global expert order, which is
what ``ZeroEngine.full_params()`` returns. The shard records are memory-mapped straight out of the
``.pt`` zips (they are stored, 64-byte aligned), so consolidating a 70B checkpoint needs host memory for
one group at a time plus the output.

    python -m distributed_llm_training_gpu_manager_amd.ckpt.zero_to_fp32 <save_dir> out.safetensors \\
        [--tag global_step120] [--dtype bf16]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from typing import Dict, Optional

import torch

from .checkpoint import MODEL0, STATE, ShardSource, complete_tags


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
    meta = torch.load(os.path.join(d, MODEL0), weights_only=True, mmap=True)
    mans = {}
    for r in meta["writers"]:
        with open(os.path.join(d, f"manifest_r{r}.json")) as f:
            mans[r] = json.load(f)
    src = ShardSource(d, mans, verify=False)
    return {k: torch.from_numpy(v).to(dtype) for k, v in src.consolidate(meta["groups"], state).items()}


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
