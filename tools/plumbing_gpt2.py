"""BASELINE config 1: GPT-2-small ZeRO-1 launched through the DeepSpeed-schema launcher on CPU/gloo,
world_size 1, loss monitor attached -> JSON summary (plumbing check, no GPU).

    python tools/plumbing_gpt2.py --out profiles/plumbing_gpt2_zero1_cpu.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_llm_training_gpu_manager_amd.launcher.config import DeepSpeedConfig, ZeROStage, OffloadDevice  # noqa
from distributed_llm_training_gpu_manager_amd.launcher.launcher import ZeroLauncher  # noqa: E402
from distributed_llm_training_gpu_manager_amd.launcher.supervisor import JobRegistry  # noqa: E402


def main(argv=None) -> dict:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--out", default=None)
    ap.add_argument("--timeout", type=float, default=900)
    a = ap.parse_args(argv)
    work = tempfile.mkdtemp(prefix="dlgm_plumbing_")
    log_json = os.path.join(work, "train.json")
    script = os.path.join(ROOT, "distributed_llm_training_gpu_manager_amd", "train.py")
    cfg = DeepSpeedConfig(model_name="gpt2-small", num_gpus=1, num_nodes=1, zero_stage=ZeROStage.OPTIMIZER_STATE,
                          offload_optimizer=OffloadDevice.NONE, offload_param=OffloadDevice.NONE,
                          train_micro_batch_size_per_gpu=1, gradient_accumulation_steps=2, bf16_enabled=True,
                          fp16_enabled=False, activation_checkpointing=False, master_port=29731)
    launcher = ZeroLauncher(registry=JobRegistry())
    t0 = time.time()
    res = launcher.launch(cfg, script, script_args=[
        "--model", "gpt2-small", "--seq-len", str(a.seq), "--steps", str(a.steps), "--device", "cpu",
        "--log-json", log_json])
    job = launcher.registry.get(res.job_id)
    while job.status not in ("succeeded", "failed", "cancelled") and time.time() - t0 < a.timeout:
        time.sleep(0.5)
    out = {"config": "GPT-2-small ZeRO-1, CPU/gloo, world_size 1, loss monitor attached (BASELINE config 1)",
           "launch": json.loads(res.model_dump_json()), "job_status": job.status, "exit_codes": job.exit_codes,
           "wall_s": round(time.time() - t0, 1)}
    if os.path.exists(log_json):
        d = json.load(open(log_json))
        out["train"] = {"steps": d["log"], "monitor": d.get("monitor"), "engine": d.get("engine")}
    with open(job.log_path) as f:
        out["log_tail"] = f.read()[-1500:]
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k not in ("log_tail",)})[:3000])
    return out


if __name__ == "__main__":
    main()
