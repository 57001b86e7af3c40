"""Local multi-process launcher (replaces ``mpirun -np N`` / the SMDDP launcher).

* one process per GPU on this node (``nproc_per_node`` defaults to all visible GPUs — SURVEY.md §2.8
  Q14: SageMaker's MPI default of one process per host would idle 7 of 8 GPUs);
* rendezvous on ``127.0.0.1:<free port>`` (torch TCPStore); multi-node jobs run the same launch on every node
  (``nnodes`` / ``node_rank`` / ``master_addr`` + a fixed port: global rank = node_rank * nproc + local rank);
* rank-prefixed, line-buffered log forwarding (rank 0 unprefixed, like the reference's rank-0 output);
* failure propagation with ``mpirun`` semantics: the first non-zero exit kills the whole group and
  its exit code becomes the launcher's.
"""
from __future__ import annotations

import os
import signal
import subprocess
import sys
import threading
import time
from typing import Dict, List, Optional, Sequence

from .smenv import build_env, free_port


def visible_gpu_count() -> int:
    """GPU count without initialising HIP in this (parent) process."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip() != ""])
    try:
        import torch

        return int(torch.cuda.device_count())
    except Exception:
        return 0


def _pump(stream, prefix: str, out) -> None:
    for line in iter(stream.readline, b""):
        try:
            out.write(prefix + line.decode(errors="replace"))
            out.flush()
        except ValueError:
            break
    stream.close()


def launch(cmd: Sequence[str], nproc: int, *, output_data_dir: str = "output/data", model_dir: str = "output/model",
           distribution: Optional[dict] = None, hyperparameters: Optional[dict] = None,
           master_port: Optional[int] = None, env_extra: Optional[Dict[str, str]] = None,
           kill_grace_s: float = 10.0, job_name: str = "local", stdout=None, nnodes: int = 1, node_rank: int = 0,
           master_addr: str = "127.0.0.1", hosts: Optional[List[str]] = None) -> int:
    """Run ``cmd`` as ``nproc`` ranks of this node; return 0 or the first failing rank's exit code.

    With ``nnodes > 1`` every node runs this with its ``node_rank`` and the same ``master_addr`` / ``master_port``
    (required: a free port cannot be agreed on locally); the world is ``nnodes * nproc`` ranks."""
    stdout = stdout or sys.stdout
    if nnodes > 1 and not master_port:
        raise ValueError("multi-node launch needs an explicit master_port shared by every node")
    if not 0 <= node_rank < nnodes:
        raise ValueError(f"node_rank {node_rank} outside [0, {nnodes})")
    port = master_port or free_port()
    hosts = hosts or ([f"algo-{i + 1}" for i in range(nnodes)])
    os.makedirs(output_data_dir, exist_ok=True)
    os.makedirs(model_dir, exist_ok=True)
    procs: List[subprocess.Popen] = []
    pumps: List[threading.Thread] = []
    ngpu = visible_gpu_count()
    for r in range(nproc):
        g = node_rank * nproc + r
        env = build_env(rank=g, local_rank=r, world_size=nnodes * nproc, local_world_size=nproc,
                        master_addr=master_addr, master_port=port, output_data_dir=output_data_dir,
                        model_dir=model_dir, num_gpus=ngpu, distribution=distribution,
                        hyperparameters=hyperparameters, job_name=job_name, hosts=hosts,
                        current_host=hosts[node_rank])
        if env_extra:
            env.update(env_extra)
        p = subprocess.Popen(list(cmd), env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                             start_new_session=True)
        procs.append(p)
        t = threading.Thread(target=_pump, args=(p.stdout, "" if g == 0 else f"[{g}] ", stdout), daemon=True)
        t.start()
        pumps.append(t)

    rc = 0
    try:
        alive = set(range(nproc))
        while alive:
            for r in list(alive):
                code = procs[r].poll()
                if code is None:
                    continue
                alive.discard(r)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    stdout.write(f"[launcher] rank {node_rank * nproc + r} exited with {code}; terminating the job\n")
                    _terminate(procs, kill_grace_s)
            time.sleep(0.05)
    except KeyboardInterrupt:
        _terminate(procs, kill_grace_s)
        rc = 130
    for t in pumps:
        t.join(timeout=5)
    return rc


def _terminate(procs: List[subprocess.Popen], grace: float) -> None:
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass
    deadline = time.time() + grace
    for p in procs:
        while p.poll() is None and time.time() < deadline:
            time.sleep(0.05)
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
            p.wait()


def maybe_self_spawn(script: str, argv: Sequence[str]) -> Optional[int]:
    """MirroredStrategy-style entry: when started bare on a multi-GPU node, re-launch as N ranks.

    Returns the job exit code if it spawned, ``None`` if the caller should run in-process.
    """
    if "RANK" in os.environ or "WORLD_SIZE" in os.environ:
        return None
    n = int(os.environ.get("HSD_NPROC", "0")) or visible_gpu_count()
    if n <= 1:
        return None
    return launch([sys.executable, "-u", os.path.abspath(script), *argv], n,
                  output_data_dir=os.environ.get("SM_OUTPUT_DATA_DIR", "output/data"),
                  model_dir=os.environ.get("SM_MODEL_DIR", "output/model"))
