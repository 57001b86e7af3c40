"""End-to-end entry logic shared by ``scripts/train.py`` and ``scripts/singe_node_train.py``.

Two batch/LR semantics, exactly as the two reference scripts differ:

* ``mode="train"`` (Horovod/SMDDP, ``scripts/train.py``): ``--train_batch_size`` is PER RANK,
  learning rate is scaled ×N (``scripts/train.py:112``), ``train_results.txt`` gets a
  ``train_runtime`` line (``:165``).
* ``mode="single_node"`` (MirroredStrategy, ``scripts/singe_node_train.py``): ``--train_batch_size``
  is the GLOBAL batch split across replicas, no LR scaling (``:78``), no runtime line (``:96-101``).

Reference fixes applied: Q3 data sharded by rank, Q4 params broadcast before
step 1, Q5 rank-0-only save + barrier, Q6 global metrics.
"""
from __future__ import annotations

import json
import logging
import os
import time
from typing import List, Optional, Sequence

import torch

from .. import data as hdata
from .. import ops
from ..models import from_pretrained, save_pretrained
from ..optim import FusedAdam
from ..parallel.ddp import resolve_compression
from ..parallel.flat_params import keep_transposed_weights
from ..parallel import FlatParamStore, GradBucketer, ShardSampler, backend, broadcast_parameters
from ..utils.args import parse_args
from ..utils.env import is_sagemaker_dp_enabled
from ..utils.logging import setup_logging
from ..utils.results_io import write_eval_results, write_train_results
from . import batch_planner
from .callbacks import FaultInjection, ModelCheckpoint, load_checkpoint, master_state_dict
from .trainer import Trainer

logger = logging.getLogger("__main__")

_DTYPES = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp8": torch.bfloat16}


def _datasets(args, cfg, tokenizer, max_len: int):
    n_train = args.num_train_examples
    n_eval = args.num_eval_examples
    if getattr(args, "task", "sequence-classification") == "masked-lm":
        if args.dataset != "synthetic":
            raise ValueError("--task masked-lm trains on --dataset synthetic (no text corpus offline)")
        tr = hdata.synthetic_mlm(n_train or 2048, max_len, cfg.vocab_size, seed=args.seed)
        te = hdata.synthetic_mlm(n_eval or 512, max_len, cfg.vocab_size, seed=args.seed + 1)
        return tr, te
    if args.dataset == "synthetic":
        tr = hdata.synthetic_classification(n_train or 2048, max_len, cfg.vocab_size, seed=args.seed,
                                            num_labels=cfg.num_labels)
        te = hdata.synthetic_classification(n_eval or 512, max_len, cfg.vocab_size, seed=args.seed + 1,
                                            num_labels=cfg.num_labels)
        return tr, te
    texts, labels = hdata.load_text_split(args.dataset, "train", args.dataset_dir)
    if n_train:
        texts, labels = texts[:n_train], labels[:n_train]
    tr = hdata.tokenize_dataset(tokenizer, texts, labels, max_len)
    texts, labels = hdata.load_text_split(args.dataset, "test", args.dataset_dir)
    if n_eval:
        texts, labels = texts[:n_eval], labels[:n_eval]
    te = hdata.tokenize_dataset(tokenizer, texts, labels, max_len)
    return tr, te


def _provenance(args, model, rank: int, n_train: int, n_eval: int, batch_plan=None) -> dict:
    """Say loudly when the run is not the reference's imdb fine-tune of pretrained weights: results files keep
    the reference's exact format, so the data / weights they came from go to ``run_provenance.json`` beside
    them and to a WARNING in the log."""
    weights = getattr(model, "weights_source", "random-init")
    synthetic = args.dataset == "synthetic"
    info = {"dataset": args.dataset, "synthetic_data": synthetic, "weights": weights,
            "model_name_or_path": args.model_name_or_path, "num_train_examples": n_train,
            "num_eval_examples": n_eval, "train_batch_size": args.train_batch_size}
    if batch_plan is not None:
        info["auto_batch"] = batch_plan.as_dict()
    if synthetic or weights == "random-init":
        what = " and ".join(x for x in (("synthetic random data" if synthetic else ""),
                                         ("random-init weights" if weights == "random-init" else "")) if x)
        logger.warning("training on %s: train_results.txt / eval_results.txt are NOT comparable with the "
                       "reference's imdb fine-tune of pretrained %s (see run_provenance.json)", what,
                       args.model_name_or_path)
    if rank == 0:
        os.makedirs(args.output_data_dir, exist_ok=True)
        with open(os.path.join(args.output_data_dir, "run_provenance.json"), "w") as f:
            json.dump(info, f, indent=1)
    return info


def build(args, mode: str):
    """Construct model/store/optimizer/bucketer/trainer for ``args``. Returns a dict of parts."""
    st = backend.init(device=args.device, timeout_s=args.dist_timeout)
    dev = st.device
    world, rank = st.world_size, st.rank
    on_gpu = dev.type == "cuda"
    dtype_name = args.dtype or ("bf16" if on_gpu else "fp32")
    compute_dtype = _DTYPES[dtype_name]
    grad_dtype = {"fp32": torch.float32, "bf16": torch.bfloat16}[args.grad_dtype or "fp32"]
    torch.manual_seed(args.seed)

    task = getattr(args, "task", "sequence-classification")
    model = from_pretrained(args.model_name_or_path or "bert-base-uncased", task=task, num_labels=args.num_labels,
                            seed=args.seed)
    model.to(dev)
    model.rng.base_seed = args.seed
    model.rng.rank = rank
    # --dtype fp8: bf16 activations / master-weight copies plus fp8 (e4m3) weight copies and per-tensor
    # quantised fp8 forward + dgrad GEMMs on the HIP path (ops/hip.py set_fp8); CPU runs stay bf16.
    if dtype_name == "fp32" and on_gpu:
        logger.info("--dtype fp32 on the GPU: the reference's precision on the fp32 kernels (ops/hip32.py: split-product "
                    "MFMA GEMMs, fp32 LayerNorm / embeddings / streaming attention / head, fused fp32 Adam); "
                    "--dtype bf16 is the fast path")
    fp8 = dtype_name == "fp8" and on_gpu and ops.hip_active(dev)
    if dtype_name == "fp8" and not fp8:
        logger.warning("--dtype fp8 needs the HIP path on a GPU; computing in bf16")
    if fp8:
        ops.set_fp8(True, getattr(args, "fp8_grad_format", "e4m3"))
    tokenizer = hdata.load_tokenizer(args.model_name_or_path, model.cfg.vocab_size, model.cfg.model_max_length)
    max_len = args.max_seq_length or min(tokenizer.model_max_length, model.cfg.max_position_embeddings)
    rank_tokens = None
    if args.train_batch_size != "auto":
        rank_tokens = (int(args.train_batch_size) // (1 if mode == "train" else world)) * max_len
    store = FlatParamStore(model, dev, compute_dtype=compute_dtype, grad_dtype=grad_dtype, fp8=fp8,
                           transposed=keep_transposed_weights(rank_tokens))
    base_lr = float(args.learning_rate)
    lr = base_lr * world if mode == "train" else base_lr  # scripts/train.py:112 vs singe_node_train.py:78
    opt = FusedAdam(store, lr=lr, eps=args.adam_epsilon, eps_mode=args.adam_eps_mode,
                    weight_decay=args.weight_decay if args.optimizer == "adamw" else 0.0)
    batch_plan = None
    if args.train_batch_size == "auto":
        # sized on the device before any readiness hook / bucketer exists (the probes are plain fwd + bwd)
        batch_plan = batch_planner.plan(model, store, max_len, dev, headroom=args.auto_batch_headroom,
                                        max_tokens=args.auto_batch_max_tokens or None,
                                        compression=resolve_compression(getattr(args, "grad_compression", "none"),
                                                                        world, on_gpu, dtype_name))
        per_gpu = batch_planner.agree_min(batch_plan.per_gpu_batch, dev)
        batch_plan.per_gpu_batch = per_gpu
        args.train_batch_size = per_gpu if mode == "train" else per_gpu * world
        logger.info("--train_batch_size auto: %d per GPU (%s, %.1f MB/sequence, fixed %.2f GB, budget %.1f of "
                    "%.1f GB, capped by %s) -> train_batch_size %d", per_gpu, batch_plan.method,
                    batch_plan.per_seq_bytes / 2**20, batch_plan.fixed_bytes / 2**30, batch_plan.budget_bytes / 2**30,
                    batch_plan.total_bytes / 2**30, batch_plan.capped_by, args.train_batch_size)
    per_rank = int(args.train_batch_size) // (1 if mode == "train" else world)
    wire = resolve_compression(getattr(args, "grad_compression", "none"), world, on_gpu, dtype_name)
    if world > 1:
        logger.info("gradient wire format: %s (--grad_compression %s)", wire, getattr(args, "grad_compression", "none"))
    bucketer = GradBucketer(store, bucket_mb=args.bucket_mb, compression=wire) if world > 1 else None
    trainer = Trainer(model, store, opt, bucketer, dev, grad_accum=args.gradient_accumulation_steps,
                      lr_schedule=getattr(args, "lr_schedule", "constant"),
                      lr_warmup_steps=getattr(args, "lr_warmup_steps", 0),
                      check_sync=args.check_sync, log_every=args.log_every, step_watchdog=args.step_watchdog,
                      hip_graph=resolve_hip_graph(getattr(args, "hip_graph", False), on_gpu, world,
                                                  per_rank * max_len, args.gradient_accumulation_steps),
                      eval_hip_graph=getattr(args, "eval_hip_graph", "auto"))
    initial_epoch = 0
    if args.resume_from:
        initial_epoch = int(load_checkpoint(args.resume_from, trainer).get("epoch", 0))
    broadcast_parameters(store, opt if args.resume_from else None)
    return {"initial_epoch": initial_epoch, "tokenizer": tokenizer, "max_len": max_len, "batch_plan": batch_plan,
            "model": model, "store": store, "optimizer": opt, "bucketer": bucketer, "trainer": trainer,
            "device": dev, "world": world, "rank": rank, "lr": lr, "dtype": dtype_name}


def resolve_hip_graph(flag, on_gpu: bool, world: int, tokens: int, accum: int) -> bool:
    """``--hip_graph``: True / False as given; ``auto`` = on for single-process GPU steps of one micro-step and at most
    HSD_GRAPH_AUTO_MAX_TOKENS (2,048) tokens, where the step is launch-bound and the replay wins (bert-base S = 128,
    one MI355X: B = 1 170-192 -> 254-261 seq/s, B = 8 1,314-1,422 -> 1,862-1,877, B = 16 3,042-3,077 -> 3,198-3,208;
    at B = 32 and bert-large B = 8 eager is 10-12 % faster: profiles/graph_small_batch_r5.log,
    profiles/graph_vs_eager_r5.log)."""
    if flag != "auto":
        return bool(flag)
    cap = int(os.environ.get("HSD_GRAPH_AUTO_MAX_TOKENS", "2048"))
    on = bool(on_gpu and world == 1 and int(accum) <= 1 and 0 < tokens <= cap)
    logger.info("--hip_graph auto: %s (%d tokens per step, cap %d, world %d)", "on" if on else "off", tokens, cap, world)
    return on


def run(argv: Optional[Sequence[str]] = None, mode: str = "train") -> dict:
    args, _unknown = parse_args(argv, "train" if mode == "train" else "single_node")
    env_rank = int(os.environ.get("RANK", "0"))
    setup_logging(env_rank)
    if mode == "train":
        logger.info(args)  # scripts/train.py:63
        if is_sagemaker_dp_enabled():
            logger.info("SMDDP requested via SM_FRAMEWORK_PARAMS: served by the RCCL data-parallel engine")
    parts = build(args, mode)
    model, trainer, dev = parts["model"], parts["trainer"], parts["device"]
    world, rank = parts["world"], parts["rank"]
    cfg = model.cfg

    tokenizer, max_len = parts["tokenizer"], parts["max_len"]
    train_ds, test_ds = _datasets(args, cfg, tokenizer, max_len)

    if mode == "train":
        per_rank_train = args.train_batch_size
    else:  # MirroredStrategy: global batch split over replicas
        if args.train_batch_size % world:
            raise ValueError(f"global train_batch_size {args.train_batch_size} not divisible by {world} replicas")
        per_rank_train = args.train_batch_size // world
    per_rank_eval = args.eval_batch_size if mode == "train" else max(1, args.eval_batch_size // world)
    # eval batch coalescing: evaluation has no dropout and no cross-example math (no batch statistics), so each
    # example's logits and loss do not depend on which examples share its forward, and the metrics are per-example
    # means (Keras evaluate with SUM_OVER_BATCH_SIZE over equal batches). Consecutive eval batches are therefore run
    # k at a time, up to --eval_coalesce_tokens tokens per forward: the reference's eval_batch_size 2 at S = 512
    # (launch.py:16) is 1,024-token forwards that leave most of the GPU idle. 0 = one forward per eval batch.
    coalesce = max(1, int(getattr(args, "eval_coalesce_tokens", 0) or 0) // max(1, per_rank_eval * max_len))
    per_rank_eval_fwd = per_rank_eval * coalesce
    if coalesce > 1:
        logger.info("evaluate: eval_batch_size %d per rank, %d batches per forward (%d sequences; "
                    "--eval_coalesce_tokens %d)", per_rank_eval, coalesce, per_rank_eval_fwd, args.eval_coalesce_tokens)

    train_loader = hdata.BatchLoader(train_ds, ShardSampler(len(train_ds), rank, world, shuffle=False, seed=args.seed,
                                                             batch_size=per_rank_train), dev)
    # eval scores every test example once (reference model.evaluate, scripts/train.py:170): shards padded with
    # ignored rows, the last partial batch kept
    test_loader = hdata.BatchLoader(test_ds, ShardSampler(len(test_ds), rank, world, shuffle=False, seed=args.seed,
                                                           drop_last=False, mark_padding=True,
                                                           batch_size=per_rank_eval_fwd), dev)
    _provenance(args, model, rank, len(train_ds), len(test_ds), parts["batch_plan"])
    out = {"args": args}
    callbacks = [FaultInjection()]
    if args.benchmark or args.profile:
        from ..obs import ProfilerCallback, ThroughputMeter

        if args.benchmark:
            callbacks.append(ThroughputMeter(args.output_data_dir, per_rank_train, max_len, warmup=args.warmup_steps,
                                             log_every=args.log_every,
                                             info={"model": args.model_name_or_path, "dtype": parts["dtype"],
                                                   "script": mode, "data": args.dataset}))
        if args.profile:
            callbacks.append(ProfilerCallback(args.output_data_dir, start=args.warmup_steps, steps=3, rank=rank))
    if args.save_every_epoch:
        callbacks.append(ModelCheckpoint(os.path.join(args.model_dir, "checkpoint-{epoch}")))

    if args.do_train:
        if mode == "train":
            logger.info("*** Train ***")
        start = time.time()
        hist = trainer.fit(train_loader, args.epochs, callbacks=callbacks, verbose=(rank == 0),
                           max_steps=args.max_steps, initial_epoch=parts["initial_epoch"])
        train_runtime = {"train_runtime": round(time.time() - start, 4)}
        if mode == "train":
            logger.info(f"train_runtime = {train_runtime}\n")
        else:
            logger.info("*** Train ***")  # singe_node_train.py logs it AFTER fit (:92)
        if rank == 0:
            write_train_results(args.output_data_dir, hist.history, train_runtime if mode == "train" else None)
        out["history"] = hist.history
        out["train_runtime"] = train_runtime

    if args.do_eval:
        logger.info("*** Evaluate ***")
        start = time.time()
        result = trainer.evaluate(test_loader)  # the meter's global all-reduce syncs the device
        eval_runtime = round(time.time() - start, 4)
        # not in eval_results.txt (the reference's writer holds the metrics only, scripts/train.py:172-179): the log line
        # and run_provenance-style JSON beside it time the reference's other measured phase, model.evaluate (:170)
        eval_speed = {"eval_runtime": eval_runtime, "eval_samples": len(test_ds),
                      "eval_samples_per_second": round(len(test_ds) / max(eval_runtime, 1e-9), 2),
                      "eval_batch_size": per_rank_eval, "eval_sequences_per_forward": per_rank_eval_fwd,
                      "eval_hip_graph": trainer.eval_graph_active}
        logger.info(f"eval_runtime = {eval_speed}")
        if rank == 0:
            write_eval_results(args.output_data_dir, result)
            with open(os.path.join(args.output_data_dir, "eval_speed.json"), "w") as f:
                json.dump(eval_speed, f, indent=1)
        out["eval"] = result
        out["eval_speed"] = eval_speed

    # Q5: rank-0-only save, then barrier
    if rank == 0:
        save_pretrained(model, args.model_dir, state_dict=master_state_dict(model, parts["store"]))
        tokenizer.save_pretrained(args.model_dir)
    backend.barrier()
    out["global_step"] = trainer.global_step
    # tear the process group down explicitly: left to interpreter exit, the c10d / gloo threads are destroyed in
    # arbitrary order and a rank can abort ("terminate called without an active exception") after a good run
    backend.shutdown()
    return out
