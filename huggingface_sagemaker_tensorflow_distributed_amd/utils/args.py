"""CLI surface of the entry scripts.

Mirrors the flags of the reference entry points (``scripts/train.py:36-52`` and
``scripts/singe_node_train.py:13-29``) with the documented fixes from SURVEY.md §2.8:

* Q1 ``--learning_rate`` is parsed as a float (the reference declares ``type=str`` and would
  compute ``"5e-5" * N`` under Horovod, ``scripts/train.py:43,112``).
* Q2 ``--do_train`` / ``--do_eval`` go through :func:`str2bool` (``type=bool`` at
  ``scripts/train.py:44-45`` cannot be switched off from the command line).
* ``SM_*`` defaults come from the environment when set, otherwise a local ``./output`` tree
  (the reference raises ``KeyError`` when the variable is missing, ``scripts/train.py:48-50``).
* Unknown flags are ignored (``parse_known_args``, ``scripts/train.py:52``).

Additive flags (benchmark / north-star knobs) never change the meaning of the reference flags.
"""
from __future__ import annotations

import argparse
import os
from typing import List, Optional, Sequence, Tuple

from .env import sm_default


def bool_or_auto(v):
    """``"auto"`` or a boolean (str2bool)."""
    if isinstance(v, str) and v.strip().lower() == "auto":
        return "auto"
    return str2bool(v)


def str2bool(v) -> bool:
    if isinstance(v, bool):
        return v
    s = str(v).strip().lower()
    if s in ("1", "true", "t", "yes", "y", "on"):
        return True
    if s in ("0", "false", "f", "no", "n", "off", "none", ""):
        return False
    raise argparse.ArgumentTypeError(f"expected a boolean, got {v!r}")


def batch_size_arg(v):
    """``--train_batch_size``: an int (the reference's ``type=int``) or ``auto`` = sized for the device's HBM
    (train/batch_planner.py)."""
    if isinstance(v, int):
        return v
    if str(v).strip().lower() == "auto":
        return "auto"
    return int(v)


def _add_reference_flags(p: argparse.ArgumentParser, *, with_n_gpus: bool) -> None:
    # scripts/train.py:39-45
    p.add_argument("--epochs", type=int, default=3)
    p.add_argument("--train_batch_size", type=batch_size_arg, default=8,
                   help="int, or 'auto': the largest per-GPU batch that fits the HBM (capped at the throughput knee)")
    p.add_argument("--eval_batch_size", type=int, default=4)
    p.add_argument("--model_name_or_path", type=str, default=None)
    p.add_argument("--learning_rate", type=float, default=5e-5)
    p.add_argument("--do_train", type=str2bool, default=True)
    p.add_argument("--do_eval", type=str2bool, default=True)
    # scripts/train.py:48-50 (SM_* environment contract)
    p.add_argument("--output_data_dir", type=str, default=sm_default("SM_OUTPUT_DATA_DIR"))
    p.add_argument("--model_dir", type=str, default=sm_default("SM_MODEL_DIR"))
    if with_n_gpus:
        p.add_argument("--n_gpus", type=str, default=sm_default("SM_NUM_GPUS"))


def _add_framework_flags(p: argparse.ArgumentParser) -> None:
    """Additive flags (SURVEY.md §2.7 'Additive flags')."""
    g = p.add_argument_group("hsd extensions")
    g.add_argument("--dtype", choices=["fp32", "bf16", "fp8"], default=None,
                   help="compute dtype (default: bf16 on GPU, fp32 on CPU)")
    g.add_argument("--max_seq_length", type=int, default=None,
                   help="pad/truncate length (default: tokenizer.model_max_length, 512 for BERT)")
    g.add_argument("--dataset", type=str, default="synthetic",
                   help="imdb | sst2 | synthetic | path to a local dataset directory/file")
    g.add_argument("--dataset_dir", type=str, default=None, help="local directory holding imdb/sst2 data")
    g.add_argument("--num_train_examples", type=int, default=None, help="synthetic/limit train size")
    g.add_argument("--num_eval_examples", type=int, default=None, help="synthetic/limit eval size")
    g.add_argument("--max_steps", type=int, default=None, help="stop each epoch after this many steps")
    g.add_argument("--seed", type=int, default=42)
    g.add_argument("--bucket_mb", type=float, default=None, help="gradient all-reduce bucket size (MiB)")
    g.add_argument("--grad_dtype", choices=["fp32", "bf16"], default=None)
    g.add_argument("--grad_compression", choices=["auto", "none", "bf16", "fp16"], default="auto",
                   help="dtype fp32 gradient buckets are all-reduced in (Horovod's hvd.Compression.fp16); auto: bf16 "
                        "for bf16 / fp8 runs on GPUs at N >= 2 (the casts cost less than the transfer time they save "
                        "over xGMI, parallel/ddp.py resolve_compression), fp32 for --dtype fp32; none = fp32 always "
                        "(the reference's Horovod all-reduce)")
    g.add_argument("--optimizer", choices=["adam", "adamw"], default="adam")
    g.add_argument("--weight_decay", type=float, default=0.0)
    g.add_argument("--adam_eps_mode", choices=["keras", "torch"], default="keras")
    g.add_argument("--adam_epsilon", type=float, default=None)
    g.add_argument("--gradient_accumulation_steps", type=int, default=1)
    g.add_argument("--lr_schedule", choices=["constant", "linear"], default="constant",
                   help="constant = Keras Adam(learning_rate) (reference); linear = warmup then linear decay to 0")
    g.add_argument("--lr_warmup_steps", type=int, default=0, help="linear warmup steps of the learning rate")
    g.add_argument("--benchmark", type=str2bool, default=False)
    g.add_argument("--warmup_steps", type=int, default=3, help="benchmark warmup steps")
    g.add_argument("--profile", type=str2bool, default=False)
    g.add_argument("--hip_graph", type=bool_or_auto, default="auto",
                   help="replay the whole step from a captured HIP graph (single-process GPU runs); auto (default) = "
                        "on for launch-bound steps of <= HSD_GRAPH_AUTO_MAX_TOKENS (2,048) tokens, one micro-step, one "
                        "process (bert-base S=128 B=1-16: 1.04-1.5x eager; B>=32: eager faster)")
    g.add_argument("--eval_hip_graph", type=bool_or_auto, default="auto",
                   help="evaluate by replaying a captured forward graph per batch shape; auto = for eval batches of <= "
                        "HSD_EVAL_GRAPH_MAX_TOKENS (16,384) tokens on the GPU (the reference's eval_batch_size 2: "
                        "launch-bound forwards)")
    g.add_argument("--eval_coalesce_tokens", type=int, default=16384,
                   help="run consecutive eval batches together, up to this many tokens per forward (metrics are "
                        "per-example: unchanged); 0 = one forward per --eval_batch_size batch")
    g.add_argument("--save_every_epoch", type=str2bool, default=False)
    g.add_argument("--resume_from", type=str, default=None)
    g.add_argument("--check_sync", type=int, default=0, help="verify cross-rank param hash every N steps")
    g.add_argument("--dist_timeout", type=float, default=1800.0, help="seconds")
    g.add_argument("--step_watchdog", type=float, default=0.0, help="abort if a step exceeds N s (0=off)")
    g.add_argument("--log_every", type=int, default=50)
    g.add_argument("--device", type=str, default=None, help="cuda | cpu (default: cuda if available)")
    g.add_argument("--num_labels", type=int, default=2)
    g.add_argument("--task", choices=["sequence-classification", "masked-lm"], default="sequence-classification",
                   help="masked-lm: RoBERTa MLM pretraining (BASELINE.json config 5)")
    g.add_argument("--auto_batch_max_tokens", type=int, default=131072,
                   help="--train_batch_size auto: cap per-GPU tokens (0 = fill the memory budget)")
    g.add_argument("--auto_batch_headroom", type=float, default=0.9,
                   help="--train_batch_size auto: fraction of the device memory the step may use")
    g.add_argument("--fp8_grad_format", choices=["e4m3", "e5m2"], default="e4m3",
                   help="--dtype fp8: format of the quantised gradients in the dgrad GEMMs")


def build_parser(script: str = "train") -> argparse.ArgumentParser:
    """``script`` is ``"train"`` (Horovod-style) or ``"single_node"`` (MirroredStrategy-style)."""
    if script not in ("train", "single_node"):
        raise ValueError(script)
    p = argparse.ArgumentParser(description=f"hsd {script} entry point")
    # scripts/singe_node_train.py:27 comments --n_gpus out; we accept it everywhere (informational)
    _add_reference_flags(p, with_n_gpus=True)
    _add_framework_flags(p)
    return p


def parse_args(argv: Optional[Sequence[str]] = None, script: str = "train") -> Tuple[argparse.Namespace, List[str]]:
    p = build_parser(script)
    args, unknown = p.parse_known_args(argv)
    return args, unknown


def hyperparameters_to_argv(hyperparameters: dict) -> List[str]:
    """SageMaker-toolkit style conversion: ``{"epochs": 1}`` -> ``["--epochs", "1"]``.

    Matches how the SageMaker training toolkit turns the estimator's ``hyperparameters``
    (``launch.py:13-18``) into entry-point argv.
    """
    out: List[str] = []
    for k, v in hyperparameters.items():
        if v is None:
            continue
        out.append(f"--{k}")
        if isinstance(v, bool):
            out.append("True" if v else "False")
        else:
            out.append(str(v))
    return out
