"""bench.py driver contract, exercised on CPU/gloo with a tiny model.

The round driver runs either ``python bench.py --gpus N ...`` or ``python -m torch.distributed.run
--nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K
--warmup W`` and reads ONE JSON line from rank 0 with a fixed set of fields; both forms of the N > 1
path (process group, max over ranks, whole-job tokens/s) are checked here with two gloo ranks, and a
rank-count mismatch must fail instead of measuring one rank.
"""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
          "vs_baseline", "dtype", "data", "config"}


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(**extra):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    env.update(extra)
    return env


def _run(cmd, **extra):
    res = subprocess.run(cmd, cwd=ROOT, env=_env(**extra), capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout
    return json.loads(lines[0])


def _check(out, n, steps, warmup):
    assert FIELDS <= set(out), FIELDS - set(out)
    assert out["n_gpus"] == n and out["steps"] == steps and out["warmup"] == warmup
    assert out["value"] > 0 and out["ms_per_step"] > 0 and out["higher_is_better"] is True
    assert out["scaling"] == "weak" and out["dtype"] == "bf16"
    cfg = out["config"]
    assert cfg["parallelism"] == f"zero3-dp{n}" and cfg["seq_len"] == 64
    # whole-job tokens/s: N ranks x mbs x seq x GA tokens per step
    tokens = n * cfg["micro_batch_per_gpu"] * cfg["seq_len"] * cfg["grad_accum"] * steps
    assert abs(out["value"] - tokens / (out["ms_per_step"] * steps / 1000)) / out["value"] < 0.02


def test_bench_single_process():
    out = _run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--model", "llama-tiny", "--seq", "64",
                "--ga", "2"])
    _check(out, 1, 2, 1)
    assert out["extra"]["comm_busbw"] is None
    # the headline metric name belongs to the headline model only; other presets name what they measured
    assert out["metric"] == "tokens/sec (node) llama-tiny ZeRO-3", out["metric"]


def test_bench_torchrun_two_ranks():
    out = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", "--steps", "2",
                "--warmup", "1", "--model", "llama-tiny", "--seq", "64", "--ga", "2"])
    _check(out, 2, 2, 1)
    assert out["extra"]["zero3_allgathers_per_step"] > 0  # partitioned: the residency plan gathers once per unit
    ops = {r["op"] for r in out["extra"]["comm_busbw"]}  # the post-timing RCCL/xGMI sweep (gloo here)
    assert ops == {"all_gather", "reduce_scatter", "all_reduce", "all_to_all"}


def test_bench_mesh_sweep_child_keeps_one_result_line():
    """--mesh-sweep on: after the result line each rank starts tools/mesh_sweep.py as a child process (a fresh
    process group on an agreed port) that first checks the transports (utils/meshcheck.py; without a GPU: the gloo
    ranks' ZeRO-3 parity against one process) and prints one [mesh-check] line; its reports go to stderr, stdout
    still holds exactly one JSON line."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", *TINY[:-2], "--comm-sweep", "off",
           "--mesh-sweep", "on"]
    res = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, res.stderr[-3000:]
    assert len([ln for ln in res.stdout.splitlines() if ln.startswith("{")]) == 1, res.stdout
    chk = [ln for ln in res.stderr.splitlines() if ln.startswith("[mesh-check] ")]
    assert len(chk) == 1, res.stderr[-3000:]
    rec = json.loads(chk[0][len("[mesh-check] "):])
    assert rec["world"] == 2 and rec["pass"], rec
    assert rec["zero3_parity"]["rccl_vs_world1"]["pass"] and "skipped" in rec["mesh_ops"]
    # the bandwidth rows need the GPU (the mesh is device memory): none on CPU
    assert not [ln for ln in res.stderr.splitlines() if ln.startswith("[mesh-sweep] ")]


TINY = ["--steps", "2", "--warmup", "1", "--model", "llama-tiny", "--seq", "64", "--ga", "2", "--comm-sweep", "off"]


def test_bench_self_launches_without_launcher():
    """`python bench.py --gpus 2` with no launcher starts torch.distributed.run itself (a child process) and
    reports a real 2-rank run -- never a silent one-rank number."""
    out = _run([sys.executable, "bench.py", "--gpus", "2", *TINY])
    _check(out, 2, 2, 1)
    assert out["extra"]["launch"] == "torchrun"
    assert out["extra"]["peak_GiB_max_over_ranks"] >= 0


def test_bench_world_size_mismatch_fails():
    res = subprocess.run([sys.executable, "bench.py", "--gpus", "2", *TINY], cwd=ROOT,
                         env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                         timeout=300)
    assert res.returncode != 0
    assert not [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert "WORLD_SIZE" in res.stderr
