"""Single-node multi-GPU fine-tuning entry point (MirroredStrategy semantics).

Same CLI as the reference ``scripts/singe_node_train.py`` (the filename typo is kept): the
``--train_batch_size`` is the GLOBAL batch split across all local GPUs and the learning rate is not
scaled (``:78``). Where the reference drives every GPU from one process with in-graph replication
(``tf.distribute.MirroredStrategy``, ``:40-41``), this script re-launches itself as one process per
GPU (RCCL all-reduce between them) when started without a launcher.
"""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

from huggingface_sagemaker_tensorflow_distributed_amd.launcher.spawn import maybe_self_spawn  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.train.runner import run  # noqa: E402


def main():
    rc = maybe_self_spawn(__file__, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    run(sys.argv[1:], mode="single_node")


if __name__ == "__main__":
    main()
