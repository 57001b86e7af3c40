"""bench.py under the driver's multi-GPU launch line, rehearsed on CPU (gloo, world 2 and 8).

The driver runs ``python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1
--master-port P bench.py --gpus N --steps K --warmup W`` and parses ONE JSON line from rank 0. Here the same line
runs 2 and 8 CPU ranks of a tiny BERT: exactly one JSON line, the contract's keys, whole-job value = global batch x
steps / time (max over ranks), DP degree in the config.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("n", [2, 8])
def test_bench_driver_line_cpu(n):
    env = dict(os.environ, OMP_NUM_THREADS="1", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", str(n),
           "--steps", "2", "--warmup", "1", "--batch_size", "2", "--seq_len", "16", "--model", "hsd-tiny-bert"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert KEYS <= set(d), set(d) ^ KEYS
    assert d["n_gpus"] == n and d["steps"] == 2 and d["warmup"] == 1
    assert d["config"]["global_batch"] == 2 * n and d["config"]["parallelism"] == f"dp{n}"
    assert d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["value"] > 0
    assert abs(d["value"] - 2 * n * 2 / (d["ms_per_step"] * 2 / 1e3)) / d["value"] < 0.01
    # self-validation after the timed loop: parameters identical on every rank, buckets in use
    v = d["validation"]
    assert v["ranks_in_sync"] is True
    assert v["n_buckets"] >= 1
    assert v["native_engine"] is False and v["rccl_world"] is None  # gloo on CPU: torch collectives
    assert v["grad_bytes_per_step"] > 0


def test_bench_exits_nonzero_when_ranks_diverge():
    """The self-validation is real: a rank whose parameters differ after the timed loop fails the job (exit 3) and
    the line says ranks_in_sync false."""
    env = dict(os.environ, OMP_NUM_THREADS="1", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               HSD_FAULT_DIVERGE_RANK="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
           "--steps", "1", "--warmup", "1", "--batch_size", "2", "--seq_len", "16", "--model", "hsd-tiny-bert"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode != 0
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and json.loads(lines[0])["validation"]["ranks_in_sync"] is False


def test_bench_refuses_gpus_world_mismatch():
    """``--gpus N`` without N ranks (WORLD_SIZE unset = 1) exits non-zero instead of printing a world-1 number."""
    env = dict(os.environ, HSD_DEVICE="cpu")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr, (r.returncode, r.stderr[-500:])
    assert r.stdout.strip() == ""
