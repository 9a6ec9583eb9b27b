#!/usr/bin/env python3
"""Headline benchmark: Llama-3-8B ZeRO-3 bf16 training tokens/sec on N MI355X GPUs of one node.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 it runs
one rank per GPU (RCCL over xGMI) under ``torch.distributed.run``. Started WITHOUT a
launcher (no ``WORLD_SIZE`` in the environment) with ``--gpus N > 1``, bench.py starts
``python -m torch.distributed.run --nproc-per-node N`` itself as a child process --
before anything touches the GPU -- relays its output and exits with its code, so the
multi-GPU number can never silently be a one-GPU number (the reference's launcher owns
the multi-process command the same way: ``/root/reference/ai_engine/deepspeed_launcher.py:277-300``).
A ``WORLD_SIZE`` that disagrees with ``--gpus`` is an error (exit 2). W untimed
warmup optimizer steps, then exactly K timed steps bracketed by a barrier +
``torch.cuda.synchronize()``; the elapsed time is the MAX over ranks; rank 0 prints
one JSON line. ``value`` is whole-job tokens/sec (all N GPUs); per-GPU work is fixed
(weak scaling). Data is synthetic (uniform random token ids), weights random-init of
the real Llama-3-8B architecture; every step draws fresh tokens (generated before the
timer starts) and runs the full forward, backward, reduce-scatter, clipping and AdamW
update. An amdsmi sampler polls this rank's GPU (junction / HBM temperature, HBM used,
power, xGMI links) on a side thread and its summary is reported in ``extra.telemetry``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "tokens/sec (node) Llama-3-8B ZeRO-3"


def _knob(v: str):
    """A ZeRO-3 residency knob from the command line: 'hbm' or a number."""
    return v if v in ("hbm", "auto") else float(v)


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _self_launch(n: int, argv) -> int:
    """Run this script under torch.distributed.run with `n` local ranks as a CHILD process (never exec:
    this process has not touched the GPU, and must not be replaced once anything has). Output is
    inherited, so rank 0's JSON line is this process's stdout; the exit code is the launcher's."""
    import signal
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__), *argv]
    print(f"[bench] no launcher: starting {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    proc = subprocess.Popen(cmd, cwd=ROOT)

    def _forward(sig, _frame):
        proc.send_signal(sig)
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, _forward)
    return proc.wait()


def _check_ranks(env, n: int) -> None:
    """After init: the process group has exactly `n` ranks and every rank drives its own device."""
    import torch.distributed as dist
    world = dist.get_world_size() if dist.is_initialized() else 1
    if world != n:
        raise SystemExit(f"[bench] error: --gpus {n} but the process group has {world} ranks")
    if world == 1:
        return
    ids = torch.tensor([env.local_rank, env.device.index if env.device.type == "cuda" else -1],
                       dtype=torch.int64, device=env.device)
    got = [torch.zeros_like(ids) for _ in range(world)]
    dist.all_gather(got, ids)
    local = [int(g[0]) for g in got]
    devs = [int(g[1]) for g in got]
    if len(set(local)) != world or (env.device.type == "cuda" and len(set(devs)) != world):
        raise SystemExit(f"[bench] error: ranks share a device (LOCAL_RANK {local}, device {devs})")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--mbs", type=int, default=1, help="micro-batch size per GPU")
    ap.add_argument("--ga", type=int, default=8, help="gradient accumulation steps (reference default 8)")
    ap.add_argument("--zero", type=int, default=3)
    ap.add_argument("--ckpt", action="store_true", help="activation checkpointing (recompute)")
    ap.add_argument("--live-params", default="hbm",
                    help="ZeRO-3 stage3_max_live_parameters: a number, or 'hbm' = sized to the GPU's memory")
    ap.add_argument("--reuse-distance", default="hbm", help="ZeRO-3 stage3_max_reuse_distance (number or 'hbm')")
    ap.add_argument("--local-grads", default="hbm",
                    help="ZeRO-2/3 gradient accumulation: 'hbm' (local fp32 + one reduce-scatter per step when the "
                         "full gradient fits in 15%% of HBM), 'on', or 'off' (reduce-scatter every micro-batch)")
    ap.add_argument("--hip-graphs", action="store_true",
                    help="replay the micro-batch loop as one captured HIP graph (1 GPU, dense models)")
    ap.add_argument("--profile-steps", type=int, default=0,
                    help="after the timed steps, trace this many extra steps with torch.profiler")
    ap.add_argument("--profile-dir", default="gpurun_out/torch_trace")
    ap.add_argument("--no-telemetry", action="store_true", help="do not poll amdsmi during the run")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"],
                    help="compute dtype (fp16: the DeepSpeed fp16 path with the dynamic loss scaler)")
    ap.add_argument("--comm-sweep", default="auto", choices=["auto", "on", "off"],
                    help="after the timed steps, measure RCCL busbw over xGMI (auto: when WORLD_SIZE > 1)")
    ap.add_argument("--comm-sweep-timeout", type=float, default=120.0)
    ap.add_argument("--mesh-sweep", default="auto", choices=["auto", "on", "off"],
                    help="after the result line, in a child process per rank: check the mesh and RCCL against each "
                         "other and one process ([mesh-check] on stderr), then on the GPU measure the device-driven "
                         "xGMI mesh collectives (auto: when WORLD_SIZE > 1 on the CPU; on GPUs only at WORLD_SIZE >= 8, the "
                         "full node -- the driver's last scaling run -- so the untried peer-mapped transport cannot "
                         "disturb the smaller runs before it)")
    ap.add_argument("--xgmi-mesh", default="off", choices=["on", "off"],
                    help="run the ZeRO collectives over the device-driven xGMI mesh instead of RCCL rings")
    ap.add_argument("--defer-expert-wgrad", default="auto", choices=["auto", "on", "off"],
                    help="MoE: expert dW once per step over the concatenated micro-batches")
    ap.add_argument("--optimizer-overlap", default="off", choices=["on", "off"],
                    help="ZeRO-3: per-group AdamW on a side stream, overlapping the next step's forward")
    ap.add_argument("--telemetry-interval", type=float, default=2.0)
    ap.add_argument("--n-layers", type=int, default=0,
                    help="override the preset's layer count (kernel profiling of big models on one GPU only; "
                         "the headline always runs the full preset)")
    args = ap.parse_args()

    # launch topology is decided before any GPU call
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            return _self_launch(args.gpus, sys.argv[1:])
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        print(f"[bench] error: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}", file=sys.stderr)
        return 2

    from distributed_llm_training_gpu_manager_amd.models import get_config
    from distributed_llm_training_gpu_manager_amd.parallel.comm import Comm, init_distributed, rccl_env
    from distributed_llm_training_gpu_manager_amd.parallel.zero import EngineConfig, ZeroEngine
    from distributed_llm_training_gpu_manager_amd import _native

    if torch.cuda.is_available() and args.gpus > torch.cuda.device_count():
        print(f"[bench] error: --gpus {args.gpus} but {torch.cuda.device_count()} GPUs are visible", file=sys.stderr)
        return 2
    env = init_distributed("cuda" if torch.cuda.is_available() else "cpu")
    _check_ranks(env, args.gpus)
    if env.device.type == "cuda":
        _native.hip_ops()  # fail loudly if the HIP kernels are not built
    comm = Comm()
    mcfg = get_config(args.model, **({"n_layers": args.n_layers} if args.n_layers else {}))
    ecfg = EngineConfig(zero_stage=args.zero, micro_batch_size=args.mbs, seq_len=args.seq, grad_accum=args.ga,
                        lr=3e-5, warmup_steps=100, total_steps=10000, grad_clip=1.0,
                        activation_checkpointing=args.ckpt, max_live_parameters=_knob(args.live_params),
                        max_reuse_distance=_knob(args.reuse_distance),
                        local_grad_accum={"on": True, "off": False}.get(args.local_grads, args.local_grads),
                        hip_graphs=args.hip_graphs, fp16=args.dtype == "fp16", xgmi_mesh=args.xgmi_mesh,
                        defer_expert_wgrad={"on": True, "off": False}.get(args.defer_expert_wgrad, "auto"),
                        optimizer_overlap=args.optimizer_overlap == "on")
    t0 = time.time()
    eng = ZeroEngine(mcfg, ecfg, env.device, comm)
    if env.device.type == "cuda":
        torch.cuda.synchronize()
    init_s = time.time() - t0

    # fresh synthetic tokens for every step (warmup and timed), drawn before any timing starts
    gen = torch.Generator(device=env.device)
    gen.manual_seed(1000 + env.rank)
    steps_data = []
    for _ in range(args.warmup + args.steps + max(0, args.profile_steps)):
        batches = []
        for _ in range(args.ga):
            toks = torch.randint(0, mcfg.vocab_size, (args.mbs, args.seq + 1), device=env.device, generator=gen)
            batches.append((toks[:, :-1].contiguous(), toks[:, 1:].contiguous()))
        steps_data.append(batches)
    telemetry = None
    if env.device.type == "cuda" and not args.no_telemetry:
        # amdsmi polling of this rank's GPU (junction / HBM temperature, HBM used, power, xGMI links)
        from distributed_llm_training_gpu_manager_amd.health.telemetry import TelemetrySampler
        telemetry = TelemetrySampler(env.device, interval_s=args.telemetry_interval).start()

    def sync():
        if env.device.type == "cuda":
            torch.cuda.synchronize()
        comm.barrier()

    for i in range(args.warmup):
        m = eng.train_step(steps_data[i])
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        m = eng.train_step(steps_data[args.warmup + i])
    sync()
    elapsed = time.perf_counter() - t0
    telem = telemetry.stop() if telemetry is not None else None
    t = torch.tensor([elapsed], dtype=torch.float64, device=env.device)
    comm.all_reduce_max(t)
    elapsed = float(t.item())
    # per-rank peak HBM, max over ranks (ZeRO-3 shards differ in size by at most one padding unit)
    peak = torch.tensor([torch.cuda.max_memory_allocated(env.device) / 1024 ** 3 if env.device.type == "cuda"
                         else 0.0], dtype=torch.float64, device=env.device)
    comm.all_reduce_max(peak)
    peak_gib = float(peak.item())

    if args.profile_steps > 0:  # outside the timed region: never part of the reported number
        from distributed_llm_training_gpu_manager_amd.utils.profiling import trace_window
        with trace_window(args.profile_dir, env.rank):
            for i in range(args.profile_steps):
                eng.train_step(steps_data[args.warmup + args.steps + i])


    tokens_per_step_gpu = args.mbs * args.seq * args.ga
    total_tokens = tokens_per_step_gpu * env.world * args.steps
    tps = total_tokens / elapsed
    flops_tok = mcfg.flops_per_token(args.seq, recompute=args.ckpt)
    tflops_gpu = tps / env.world * flops_tok / 1e12
    loss = float(m["loss"])
    mcfg_label = args.model + (f" ({args.n_layers} layers)" if args.n_layers else "")
    out = None
    if env.rank == 0:
        out = {
            # the headline metric name only for the headline model; other presets say what they measured
            "metric": METRIC if args.model == "llama3-8b" and not args.n_layers else
            f"tokens/sec (node) {mcfg_label} ZeRO-{args.zero}",
            "value": round(tps, 2),
            "unit": "tokens/s",
            "n_gpus": env.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1000, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (uniform random token ids; random-init weights)",
            "config": {
                "model": mcfg.name if not args.n_layers else f"{mcfg.name} ({mcfg.n_layers} layers)",
                "global_batch": args.mbs * args.ga * env.world,
                "micro_batch_per_gpu": args.mbs,
                "grad_accum": args.ga,
                "seq_len": args.seq,
                "parallelism": f"zero{args.zero}-dp{env.world}",
                "activation_checkpointing": args.ckpt,
                "stage3_max_live_parameters": args.live_params,
                "stage3_max_reuse_distance": args.reuse_distance,
                "grad_reduce_scatter": ("none (single rank)" if eng.W == 1 else
                                        "per_step" if eng.local_grads else "per_micro_batch"),
                "hip_graphs": eng._graph is not None,
                "transport": ("xgmi_mesh" if eng.mesh is not None else "rccl") if eng.W > 1 else "none",
                "step_reduce_dtype": str(ecfg.step_comm_dtype).replace("torch.", "") if eng.local_grads else None,
            },
            "extra": {
                "tokens_per_sec_per_gpu": round(tps / env.world, 2),
                "model_tflops_per_gpu": round(tflops_gpu, 1),
                "mfu_vs_2.5PF_dense_bf16": round(tflops_gpu / 2500.0, 4),
                "final_loss": round(loss, 4),
                "final_grad_norm": round(float(m["grad_norm"]), 4),
                "init_s": round(init_s, 1),
                "params": eng.num_params(),
                "zero3_allgathers_per_step": eng.live_plan.gathers_per_step(args.ga),
                "zero3_resident_gathered_params": eng.live_plan.resident_params,
                "mem": {k: round(v, 1) for k, v in eng.memory_report().items()},
                "peak_GiB_max_over_ranks": round(peak_gib, 1),
                "launch": "torchrun" if "TORCHELASTIC_RUN_ID" in os.environ else "single process",
                "telemetry": telem,
                "comm_busbw": None,
                "comm_env": rccl_env(apply=False) if env.backend == "nccl" else None,
            },
        }
    if args.comm_sweep == "on" or (args.comm_sweep == "auto" and env.world > 1):
        # outside the timed region: the xGMI bus-bandwidth curve of this node at this world size (ring
        # collectives and the direct mesh all-gather). A watchdog on every rank prints the result line
        # without the curve and ends the process if the sweep stalls, so the measurement is never lost.
        import threading
        from distributed_llm_training_gpu_manager_amd.utils.commbench import sweep

        def _stalled():
            if out is not None:
                out["extra"]["comm_busbw"] = "sweep timed out"
                print(json.dumps(out), flush=True)
            os._exit(0)
        dog = threading.Timer(args.comm_sweep_timeout, _stalled)
        dog.daemon = True
        dog.start()
        try:  # a failing collective must never cost the result line
            rows = sweep(comm, env.device, sizes_mb=(16, 64, 256) if env.device.type == "cuda" else (1,))
        except Exception as e:  # noqa: BLE001
            rows = f"sweep failed: {type(e).__name__}: {e}"[:400]
        dog.cancel()
        if out is not None:
            out["extra"]["comm_busbw"] = rows
    mesh_sweep = args.mesh_sweep == "on" or (args.mesh_sweep == "auto" and env.world > 1 and
                                              (env.device.type != "cuda" or env.world >= 8))
    port = None
    if mesh_sweep and env.world > 1:  # agree on the child job's rendezvous port while the group still exists
        pt = torch.tensor([_free_port() if env.rank == 0 else 0], dtype=torch.int64, device=env.device)
        torch.distributed.broadcast(pt, src=0)
        port = int(pt.item())
    if out is not None:
        print(json.dumps(out), flush=True)
    for m_ in (eng.mesh, eng.ep_mesh):
        if m_ is not None:
            m_.close()  # collective: every rank unmaps its peers' heaps before any heap is freed
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()
    if mesh_sweep:
        _mesh_sweep_child(port, eng, args.comm_sweep_timeout)
    return 0


def _mesh_sweep_child(port, eng, timeout_s: float) -> None:
    """The ipc_mesh_* bus-bandwidth rows in a child process per rank, after the result line is out (VERDICT r3:
    a new transport must never share the measuring process). Its output goes to stderr; stdout keeps one line."""
    import gc
    import subprocess
    eng.__dict__.clear()  # hand this rank's HBM back before the child maps its heaps
    gc.collect()
    if torch.cuda.is_available():
        torch.cuda.empty_cache()
    env = dict(os.environ)
    # the child job hosts its own rendezvous store (rank 0 serves it on the agreed port): not torchrun's agent store
    env.pop("TORCHELASTIC_USE_AGENT_STORE", None)
    if port is not None:
        env["MASTER_PORT"] = str(port)
    if os.path.isdir(os.path.join(ROOT, "gpurun_out")):
        env.setdefault("DLGM_SWEEP_DIR", os.path.join(ROOT, "gpurun_out"))
    try:
        subprocess.run([sys.executable, os.path.join(ROOT, "tools", "mesh_sweep.py")], env=env, cwd=ROOT,
                       stdout=sys.stderr, stderr=sys.stderr, timeout=timeout_s)
    except Exception as e:  # noqa: BLE001 -- the result line is already out
        print(f"[bench] mesh sweep: {type(e).__name__}: {e}", file=sys.stderr, flush=True)


if __name__ == "__main__":
    sys.exit(main())
