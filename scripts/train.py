"""Multi-process data-parallel fine-tuning entry point (Horovod/SMDDP semantics).

Same CLI and outputs as the reference ``scripts/train.py`` (flags ``:38-50``, results
``:157-179``, save ``:182-183``); runs one process per GPU under ``launch.py`` /
``python -m huggingface_sagemaker_tensorflow_distributed_amd.launcher`` / ``torchrun``.
"""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

from huggingface_sagemaker_tensorflow_distributed_amd.train.runner import run  # noqa: E402


def main():
    run(sys.argv[1:], mode="train")


if __name__ == "__main__":
    main()
