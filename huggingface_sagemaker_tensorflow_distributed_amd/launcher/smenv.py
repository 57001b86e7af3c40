"""SageMaker-container environment emulation (reference L1, SURVEY.md §2.7 'Environment contract').

The SageMaker training toolkit writes ``SM_*`` variables and turns the estimator's hyperparameters
into argv before starting the entry point (``launch.py:36-55`` → container). The local launcher
does the same for each rank, plus torchrun-style rank variables.
"""
from __future__ import annotations

import json
import os
import socket
from typing import Dict, List, Optional, Tuple


def free_port() -> int:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def distribution_flags(distribution: Optional[dict]) -> Dict[str, bool]:
    """Map the estimator ``distribution`` dict (``launch.py:20-24``) to SM_FRAMEWORK_PARAMS flags."""
    d = distribution or {}
    smddp = bool(d.get("smdistributed", {}).get("dataparallel", {}).get("enabled", False))
    mpi = bool(d.get("mpi", {}).get("enabled", False))
    torch_dist = bool(d.get("torch_distributed", {}).get("enabled", False))
    return {"sagemaker_distributed_dataparallel_enabled": smddp, "sagemaker_mpi_enabled": mpi,
            "sagemaker_torch_distributed_enabled": torch_dist}


def node_topology(instance_count: int = 1) -> Tuple[List[str], int]:
    """(hosts, this node's index) of a multi-node job, from the SageMaker container contract (``SM_HOSTS`` JSON
    list + ``SM_CURRENT_HOST``; the first host is the rendezvous master) or ``HSD_HOSTS`` (comma list) +
    ``HSD_NODE_RANK``. One node without either."""
    hosts_json = os.environ.get("SM_HOSTS")
    if hosts_json and os.environ.get("SM_CURRENT_HOST"):
        hosts = list(json.loads(hosts_json))
        return hosts, hosts.index(os.environ["SM_CURRENT_HOST"])
    if os.environ.get("HSD_HOSTS"):
        hosts = [h.strip() for h in os.environ["HSD_HOSTS"].split(",") if h.strip()]
        return hosts, int(os.environ.get("HSD_NODE_RANK", "0"))
    if instance_count > 1:
        raise ValueError(f"instance_count={instance_count}: run the same launch on every node with SM_HOSTS / "
                         "SM_CURRENT_HOST (or HSD_HOSTS / HSD_NODE_RANK) set; the first host is the master")
    return ["algo-1"], 0


def build_env(*, rank: int, local_rank: int, world_size: int, local_world_size: int, master_addr: str,
              master_port: int, output_data_dir: str, model_dir: str, num_gpus: int,
              distribution: Optional[dict] = None, hyperparameters: Optional[dict] = None,
              base: Optional[Dict[str, str]] = None, job_name: str = "local",
              hosts: Optional[List[str]] = None, current_host: Optional[str] = None) -> Dict[str, str]:
    env = dict(os.environ if base is None else base)
    hosts = hosts or ["algo-1"]
    env.update({
        "RANK": str(rank), "LOCAL_RANK": str(local_rank), "WORLD_SIZE": str(world_size),
        "LOCAL_WORLD_SIZE": str(local_world_size), "MASTER_ADDR": master_addr, "MASTER_PORT": str(master_port),
        "SM_OUTPUT_DATA_DIR": output_data_dir, "SM_MODEL_DIR": model_dir, "SM_NUM_GPUS": str(num_gpus),
        "SM_CURRENT_HOST": current_host or hosts[0], "SM_HOSTS": json.dumps(hosts), "SM_TRAINING_ENV": json.dumps(
            {"job_name": job_name, "hyperparameters": hyperparameters or {}}),
        "SM_HPS": json.dumps(hyperparameters or {}),
        "SM_FRAMEWORK_PARAMS": json.dumps(distribution_flags(distribution)),
        # dmabuf IPC only on this host driver (RCCL / CUDA-tensor sharing needs it)
        "HSA_ENABLE_IPC_MODE_LEGACY": env.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
        "PYTHONUNBUFFERED": "1",
    })
    for k, v in (hyperparameters or {}).items():
        env[f"SM_HP_{str(k).upper()}"] = str(v)
    return env
