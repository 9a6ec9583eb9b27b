#!/usr/bin/env python3
"""Round 6: Mixtral 2-layer bench A/B -- VARIANT=nowt: no cached expert-weight transposes (the grouped dX GEMMs read
the [E, out, in] weights MN-contiguous instead of a per-step rebuilt [E, in, out] copy). Runs bench.py's main."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from distributed_llm_training_gpu_manager_amd.parallel import zero as Z  # noqa: E402

v = os.environ.get("VARIANT", "")
if v == "nowt":
    orig = Z.ZeroEngine.__init__

    def init(self, model_cfg, cfg, *a, **k):
        cfg.expert_weight_cache = False
        orig(self, model_cfg, cfg, *a, **k)
    Z.ZeroEngine.__init__ = init
elif v == "nohead":  # (round-6 experiment, since removed) the LM head's dW per micro-batch, not once per step
    orig = Z.ZeroEngine.__init__

    def init(self, model_cfg, cfg, *a, **k):
        cfg.defer_head_wgrad = False
        orig(self, model_cfg, cfg, *a, **k)
    Z.ZeroEngine.__init__ = init
elif v == "tcmain":  # the per-step W^T rebuild on the compute stream instead of the "tcache" side stream
    from distributed_llm_training_gpu_manager_amd.utils import streams as S
    _side = S.side_stream
    S.side_stream = lambda device, name: None if name == "tcache" else _side(device, name)
import bench  # noqa: E402

sys.argv = ["bench.py", "--model", "mixtral-8x7b", "--n-layers", "2", "--seq", "4096", "--ga", "4", "--steps", "15",
            "--warmup", "3", "--no-telemetry"]
if v == "ovl":  # per-group AdamW on the optimizer stream beside the next step's forward
    sys.argv += ["--optimizer-overlap", "on"]
sys.exit(bench.main())
