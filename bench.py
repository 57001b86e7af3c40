"""Headline benchmark: whole-node sequences/sec, BERT-base seq_len 128, bf16, DP over RCCL.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 launched by
``torch.distributed.run`` with one rank per GPU. W untimed warmup steps, then EXACTLY K timed full
training steps (forward + backward + bucketed all-reduce + fused Adam), bracketed by barrier +
device synchronize on both sides; the max over ranks is reported. Rank 0 prints ONE JSON line.

Data: synthetic full-length sequences of the reference's tensor shapes (offline box, no IMDB);
weights: random-init bert-base-uncased architecture (no hub). Dropout on, as in training.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from huggingface_sagemaker_tensorflow_distributed_amd import data as hdata  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.parallel import backend, rccl_env  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.parallel.collectives import params_in_sync  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.train.runner import build  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.utils.args import batch_size_arg, bool_or_auto, build_parser  # noqa: E402

METRIC = "sequences/sec (whole node) BERT-base seq128 at 1/2/4/8 MI355X"
BASELINE_VALUE = None  # the reference publishes no number


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch_size", type=batch_size_arg, default=batch_size_arg(os.environ.get("HSD_BENCH_BATCH", "1024")),
                    help="per-GPU batch, or 'auto' (sized for the device memory, train/batch_planner.py)")
    ap.add_argument("--auto_batch_max_tokens", type=int, default=131072,
                    help="--batch_size auto: per-GPU token cap (0 = fill the HBM budget)")
    ap.add_argument("--seq_len", type=int, default=128)
    ap.add_argument("--model", default="bert-base-uncased")
    ap.add_argument("--bucket_mb", type=float, default=None)
    ap.add_argument("--grad_dtype", default=None)
    ap.add_argument("--dtype", choices=["bf16", "fp8", "fp32"], default="bf16",
                    help="fp8: fp8 forward/dgrad GEMMs (secondary config; the headline is bf16); fp32: the reference's "
                         "own precision (scripts/train.py:113-123 sets no mixed-precision policy) on the fp32 kernels "
                         "of ops/hip32.py")
    ap.add_argument("--task", choices=["sequence-classification", "masked-lm"], default="sequence-classification")
    ap.add_argument("--hip_graph", type=bool_or_auto, default="auto",
                    help="replay the whole step from a captured HIP graph (N=1); auto = the CLI's rule (launch-bound "
                         "steps of <= 2,048 tokens only: off for the headline's 131,072)")
    a = ap.parse_args()

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus != world_env:
        # a world-1 number printed for `--gpus 8` would be recorded as the 8-GPU point of the scaling curve
        print(f"bench: --gpus {a.gpus} but WORLD_SIZE={world_env}: launch N ranks with torch.distributed.run "
              f"--nproc-per-node {a.gpus}", file=sys.stderr, flush=True)
        sys.exit(2)
    targs, _ = build_parser("train").parse_known_args(
        ["--model_name_or_path", a.model, "--train_batch_size", str(a.batch_size), "--dtype", a.dtype,
         "--task", a.task, "--hip_graph", str(a.hip_graph),
         "--learning_rate", "5e-5", "--log_every", "0", "--max_seq_length", str(a.seq_len),
         "--auto_batch_max_tokens", str(a.auto_batch_max_tokens)]
        + (["--bucket_mb", str(a.bucket_mb)] if a.bucket_mb else [])
        + (["--grad_dtype", a.grad_dtype] if a.grad_dtype else []))
    parts = build(targs, "train")
    trainer, dev, world, rank = parts["trainer"], parts["device"], parts["world"], parts["rank"]
    cfg = parts["model"].cfg
    a.batch_size = targs.train_batch_size  # resolved when --batch_size auto
    n_batches = 4
    if a.task == "masked-lm":
        ds = hdata.synthetic_mlm(a.batch_size * n_batches, a.seq_len, cfg.vocab_size, seed=1234 + rank)
    else:
        ds = hdata.synthetic_classification(a.batch_size * n_batches, a.seq_len, cfg.vocab_size,
                                            seed=1234 + rank, full_length=True)
    batches = []
    for i in range(n_batches):
        sl = slice(i * a.batch_size, (i + 1) * a.batch_size)
        batches.append({"input_ids": torch.from_numpy(ds.input_ids[sl]).long().to(dev),
                        "attention_mask": torch.from_numpy(ds.attention_mask[sl]).long().to(dev),
                        "labels": torch.from_numpy(ds.labels[sl]).long().to(dev)})

    def sync():
        backend.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    for i in range(a.warmup):
        trainer.train_step([batches[i % n_batches]])
    sync()
    t0 = time.perf_counter()
    for i in range(a.steps):
        trainer.train_step([batches[i % n_batches]])
    sync()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if backend.is_distributed():
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    dt = float(t.item())
    ms = dt * 1e3 / a.steps
    # comm/compute overlap of one extra, untimed step (native RCCL engine only): per-bucket HIP events
    overlap = None
    buck = trainer.bucketer
    if buck is not None and buck.set_timing(True):
        trainer.train_step([batches[0]])
        overlap = buck.overlap_report()
        buck.set_timing(False)
        if overlap is not None:
            overlap.pop("buckets", None)
    value = a.batch_size * world * a.steps / dt
    # untimed self-validation (the driver's N > 1 runs): every rank ends the timed steps with bit-identical
    # parameters, and the gradient path really spans the job (native RCCL engine of `world` ranks, its buckets)
    div = os.environ.get("HSD_FAULT_DIVERGE_RANK")  # test hook: perturb one rank's weights after the timed steps
    if div is not None and int(div) == rank:
        with torch.no_grad():
            trainer.store.master[0] += 1e-3
    in_sync = params_in_sync(trainer.store)
    engine = getattr(trainer.bucketer, "engine", None)
    rccl_world = int(engine.world) if engine is not None else None
    validation = {"ranks_in_sync": in_sync, "rccl_world": rccl_world, "native_engine": engine is not None,
                  "n_buckets": len(trainer.bucketer.buckets) if trainer.bucketer is not None else 0,
                  "grad_bytes_per_step": trainer.store.grad.numel() * trainer.store.grad.element_size()
                  if world > 1 else 0}
    if world > 1:
        validation["rccl_env"] = rccl_env.effective()
    ok = in_sync and (engine is None or rccl_world == world)
    if rank == 0:
        print(json.dumps({
            "metric": METRIC, "value": round(value, 2), "unit": "sequences/sec", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": (value / BASELINE_VALUE) if BASELINE_VALUE else None,
            "dtype": a.dtype, "data": "synthetic (random-init weights, full-length seq, dropout on)",
            "config": {"model": a.model, "task": a.task, "global_batch": a.batch_size * world,
                       "per_gpu_batch": a.batch_size,
                       "seq_len": a.seq_len, "parallelism": f"dp{world}",
                       "ops": "torch-reference" if os.environ.get("HSD_OPS") == "torch" else "hip",
                       "hip_graph": trainer._seed is not None,
                       "grad_wire": trainer.bucketer.compression if trainer.bucketer is not None else None,
                       "comm": ("native-rccl" if getattr(trainer.bucketer, "engine", None) is not None
                                else ("torch-" + backend.state().backend if world > 1 else "none"))},
            "validation": validation,
            **({"comm_overlap": overlap} if overlap is not None else {}),
            **({"batch_plan": parts["batch_plan"].as_dict()} if parts.get("batch_plan") is not None else {}),
        }), flush=True)
    backend.shutdown()
    if not ok:
        print(f"bench: rank {rank}: validation failed {validation}", file=sys.stderr, flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
