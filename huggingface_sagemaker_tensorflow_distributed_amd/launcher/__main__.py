"""``python -m huggingface_sagemaker_tensorflow_distributed_amd.launcher --nproc-per-node N script.py [args]``

torchrun-style local launcher with the SageMaker env contract and mpirun failure semantics.
"""
from __future__ import annotations

import argparse
import sys

from .spawn import launch, visible_gpu_count


def main(argv=None) -> int:
    p = argparse.ArgumentParser(prog="hsd-launch")
    p.add_argument("--nproc-per-node", "--nproc_per_node", type=int, default=0)
    p.add_argument("--master-port", type=int, default=0)
    p.add_argument("--output-data-dir", default="output/data")
    p.add_argument("--model-dir", default="output/model")
    p.add_argument("script")
    p.add_argument("script_args", nargs=argparse.REMAINDER)
    a = p.parse_args(argv)
    n = a.nproc_per_node or max(1, visible_gpu_count())
    return launch([sys.executable, "-u", a.script, *a.script_args], n, output_data_dir=a.output_data_dir,
                  model_dir=a.model_dir, master_port=a.master_port or None)


if __name__ == "__main__":
    sys.exit(main())
