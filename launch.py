"""Job launcher with the same shape as the reference ``launch.py``.

Reference (``launch.py:1-55``): AWS session + IAM role, a ``hyperparameters`` dict, a
``distribution`` selector (SMDDP / Horovod-MPI / None), instance type/count, then
``HuggingFace(...).fit()`` which runs ``scripts/train.py`` on SageMaker. Here the estimator runs the
same entry point on THIS node: one rank per MI355X over RCCL/xGMI (no AWS, no image).

    python launch.py                      # distribution=None -> 1 process (reference default)
    HSD_DISTRIBUTION=smddp python launch.py   # all local GPUs, one rank each
"""
import os

from huggingface_sagemaker_tensorflow_distributed_amd.launcher import HuggingFace

# hyperparameters, which are passed into the training job (launch.py:13-18)
hyperparameters = {
    "epochs": 1,
    "train_batch_size": 8,
    "eval_batch_size": 2,
    "model_name_or_path": "bert-large-uncased-whole-word-masking",
    # additive knobs (offline box: synthetic data / random-init weights unless a local dir is given)
    "dataset": os.environ.get("HSD_DATASET", "synthetic"),
    "max_steps": int(os.environ.get("HSD_MAX_STEPS", "20")),
    "num_train_examples": int(os.environ.get("HSD_NUM_TRAIN", "2048")),
    "num_eval_examples": int(os.environ.get("HSD_NUM_EVAL", "256")),
    # None = the CLI default (bf16 on a GPU); "fp32" = the reference's own precision
    "dtype": os.environ.get("HSD_DTYPE"),
    "eval_hip_graph": os.environ.get("HSD_EVAL_HIP_GRAPH"),  # None = auto (captured forwards at eval batch 2)
    "do_train": os.environ.get("HSD_DO_TRAIN"),
    "eval_coalesce_tokens": os.environ.get("HSD_EVAL_COALESCE_TOKENS"),  # None = 16,384 tokens per eval forward
}
# configuration for running training on smdistributed Data Parallel -> RCCL DP engine
# distribution = {'smdistributed': {'dataparallel': {'enabled': True}}}
# horovod launch -> RCCL DP engine
# distribution = {"mpi": {"enabled": True, "custom_mpi_options": "-verbose --NCCL_DEBUG=INFO"}}
# no distribution
distribution = {
    "smddp": {"smdistributed": {"dataparallel": {"enabled": True}}},
    "mpi": {"mpi": {"enabled": True}},
    "none": None,
}[os.environ.get("HSD_DISTRIBUTION", "none")]
# instance configurations: "mi355x" = every local GPU
instance_type = os.environ.get("HSD_INSTANCE_TYPE", "mi355x")
# multi-node: set HSD_INSTANCE_COUNT and, on every node, SM_HOSTS / SM_CURRENT_HOST (or HSD_HOSTS / HSD_NODE_RANK)
instance_count = int(os.environ.get("HSD_INSTANCE_COUNT", "1"))

huggingface_estimator = HuggingFace(
    # distributed script,
    entry_point="train.py",
    # single_node script,
    # entry_point="singe_node_train.py",
    source_dir=os.path.join(os.path.dirname(os.path.abspath(__file__)), "scripts"),
    instance_type=instance_type,
    instance_count=instance_count,
    distribution=distribution,
    hyperparameters=hyperparameters,
    base_job_name="hf-tf-bert-" + str(instance_count) + "node-" + instance_type.replace(".", "-"),
    debugger_hook_config=False,
)

if __name__ == "__main__":
    huggingface_estimator.fit()
