"""``python -m huggingface_sagemaker_tensorflow_distributed_amd.launcher --nproc-per-node N script.py [args]``

torchrun-style launcher with the SageMaker env contract and mpirun failure semantics. Multi-node: run the same
command on every node with ``--nnodes K --node-rank i --master-addr <node 0> --master-port P``.
"""
from __future__ import annotations

import argparse
import sys

from .spawn import launch, visible_gpu_count


def main(argv=None) -> int:
    p = argparse.ArgumentParser(prog="hsd-launch")
    p.add_argument("--nproc-per-node", "--nproc_per_node", type=int, default=0)
    p.add_argument("--master-port", type=int, default=0)
    p.add_argument("--nnodes", type=int, default=1)
    p.add_argument("--node-rank", "--node_rank", type=int, default=0)
    p.add_argument("--master-addr", default="127.0.0.1", help="rendezvous host (node 0) of a multi-node job")
    p.add_argument("--output-data-dir", default="output/data")
    p.add_argument("--model-dir", default="output/model")
    p.add_argument("script")
    p.add_argument("script_args", nargs=argparse.REMAINDER)
    a = p.parse_args(argv)
    n = a.nproc_per_node or max(1, visible_gpu_count())
    return launch([sys.executable, "-u", a.script, *a.script_args], n, output_data_dir=a.output_data_dir,
                  model_dir=a.model_dir, master_port=a.master_port or None, nnodes=a.nnodes, node_rank=a.node_rank,
                  master_addr=a.master_addr)


if __name__ == "__main__":
    sys.exit(main())
