"""``HuggingFace``-estimator look-alike that runs the job on THIS node.

Reference L0 (``launch.py:36-55``): ``HuggingFace(entry_point, source_dir, instance_type,
instance_count, distribution, hyperparameters, base_job_name, ...)`` then ``.fit()`` with no input
channels. Here ``.fit()`` converts hyperparameters to argv, emulates the SageMaker ``SM_*`` contract
and spawns one rank per GPU (or one process for ``distribution=None`` on a single GPU, like the
reference's ``ml.p3.2xlarge`` default), blocking and streaming logs like the SDK does.

AWS-only arguments (``role``, ``session``, ``image_uri``, ``py_version``, ``transformers_version``,
``tensorflow_version``, ``debugger_hook_config``, ``volume_size``) are accepted and recorded so an
unmodified launch script runs; they have no local meaning.
"""
from __future__ import annotations

import datetime
import logging
import os
import sys
from typing import Dict, Optional

from ..utils.args import hyperparameters_to_argv
from .smenv import node_topology
from .spawn import launch, visible_gpu_count

logger = logging.getLogger(__name__)

# instance -> GPUs per node, for the instance types the reference names (launch.py:26-28)
INSTANCE_GPUS = {
    "ml.p3.2xlarge": 1, "ml.p3.8xlarge": 4, "ml.p3.16xlarge": 8, "ml.p3dn.24xlarge": 8,
    "ml.p4d.24xlarge": 8, "local": None, "local_gpu": None, "mi355x": None, "mi355x.8x": 8,
}


class LocalEstimator:
    def __init__(self, entry_point: str, source_dir: str = ".", hyperparameters: Optional[Dict] = None,
                 distribution: Optional[Dict] = None, instance_type: str = "local", instance_count: int = 1,
                 base_job_name: Optional[str] = None, nproc_per_node: Optional[int] = None,
                 output_path: str = "output", **aws_kwargs):
        # multi-node (instance_count > 1): the same estimator runs on every node; the node list and this node's
        # index come from the SageMaker container contract (SM_HOSTS / SM_CURRENT_HOST) or HSD_HOSTS / HSD_NODE_RANK
        self._hosts, self._node_rank = node_topology(instance_count)
        if instance_count != len(self._hosts):
            raise ValueError(f"instance_count={instance_count} but {len(self._hosts)} host(s) in the environment")
        self.entry_point = entry_point
        self.source_dir = source_dir
        self.hyperparameters = dict(hyperparameters or {})
        self.distribution = distribution
        self.instance_type = instance_type
        self.instance_count = instance_count
        self.base_job_name = base_job_name or "hsd-job"
        self.output_path = output_path
        self.aws_kwargs = aws_kwargs
        self._nproc = nproc_per_node
        self.latest_job_name: Optional[str] = None
        self.model_data: Optional[str] = None

    def nproc(self) -> int:
        if self._nproc:
            return int(self._nproc)
        gpus = visible_gpu_count()
        want = INSTANCE_GPUS.get(self.instance_type)
        if self.distribution is None:
            # distribution=None: one process (launch.py:24); singe_node_train.py self-spawns its replicas
            return 1
        n = want if want is not None else gpus
        return max(1, min(n, gpus) if gpus else 1)

    def job_name(self) -> str:
        ts = datetime.datetime.now().strftime("%Y-%m-%d-%H-%M-%S-%f")[:-3]
        return f"{self.base_job_name}-{ts}"

    def fit(self, inputs=None, wait: bool = True, job_name: Optional[str] = None) -> int:
        if inputs:
            logger.warning("input channels are not used: data is read locally by the entry point")
        name = job_name or self.job_name()
        self.latest_job_name = name
        out_root = os.path.join(self.output_path, name)
        data_dir = os.path.join(out_root, "output", "data")
        model_dir = os.path.join(out_root, "model")
        script = os.path.join(self.source_dir, self.entry_point)
        cmd = [sys.executable, "-u", script, *hyperparameters_to_argv(self.hyperparameters)]
        n = self.nproc()
        logger.info("job %s: %d process(es) running %s", name, n, " ".join(cmd))
        nnodes = len(self._hosts)
        rc = launch(cmd, n, output_data_dir=data_dir, model_dir=model_dir, distribution=self.distribution,
                    hyperparameters=self.hyperparameters, job_name=name, nnodes=nnodes, node_rank=self._node_rank,
                    master_addr=self._hosts[0] if nnodes > 1 else "127.0.0.1",
                    master_port=int(os.environ.get("HSD_MASTER_PORT", "29500")) if nnodes > 1 else None,
                    hosts=self._hosts if nnodes > 1 else None)
        self.model_data = model_dir
        if rc != 0:
            raise RuntimeError(f"training job {name} failed with exit code {rc}")
        return rc


# the reference constructs `HuggingFace(...)` (launch.py:36); same name, local semantics
HuggingFace = LocalEstimator
