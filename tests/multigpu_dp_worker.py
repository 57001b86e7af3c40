"""Worker of tests/test_multigpu.py (not collected by pytest): a few native-engine DP training steps of a small BERT.

    python -m torch.distributed.run --nproc-per-node N tests/multigpu_dp_worker.py OUT   (DP over N GPUs, RCCL engine)
    python tests/multigpu_dp_worker.py OUT                                              (one process, global batch)

Every rank trains on its rank-strided share of the same global batches (dropout off); rank 0 writes the first step's
gradient (the all-reduced SUM / world = the gradient of the global-batch mean loss), the parameters after all steps,
whether every rank holds identical parameters, and what the gradient path ran on."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model, resolve_config  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.optim import FusedAdam  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore, GradBucketer, backend  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.parallel.collectives import (broadcast_parameters,  # noqa: E402
                                                                                   params_in_sync)
from huggingface_sagemaker_tensorflow_distributed_amd.train.trainer import Trainer  # noqa: E402

GLOBAL_B, S, STEPS = 8, 128, 3


def main(out):
    st = backend.init(device="cuda")
    dev, world, rank = st.device, st.world_size, st.rank
    cfg = resolve_config("hsd-tiny-bert").replace(hidden_size=256, num_attention_heads=4, intermediate_size=512,
                                                  hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    model = build_model(cfg, seed=0).to(dev)
    store = FlatParamStore(model, dev, compute_dtype=torch.bfloat16)
    opt = FusedAdam(store, lr=1e-3)
    # HSD_MGPU_COMPRESSION=fp16|bf16: 16-bit gradient wire (Horovod's Compression.fp16); HSD_MGPU_GRAPH=1: the whole
    # step captured once and replayed (train/graph.py; data parallel needs HSD_GRAPH_DP=1)
    comp = os.environ.get("HSD_MGPU_COMPRESSION", "none")
    buck = GradBucketer(store, bucket_mb=1.0, compression=comp) if world > 1 else None
    tr = Trainer(model, store, opt, buck, dev, hip_graph=os.environ.get("HSD_MGPU_GRAPH", "0") == "1")
    tr.zero_grad_in_optimizer = False  # the first step's reduced gradient is read back after the step
    if world > 1:
        broadcast_parameters(store, opt)
    g = torch.Generator().manual_seed(1234)
    first_grad = None
    for step in range(STEPS):
        ids = torch.randint(5, cfg.vocab_size, (GLOBAL_B, S), generator=g)
        am = torch.ones(GLOBAL_B, S, dtype=torch.long)
        am[1::3, S // 2:] = 0
        labels = torch.randint(0, 2, (GLOBAL_B,), generator=g)
        sl = slice(rank, GLOBAL_B, world)
        batch = {"input_ids": ids[sl].to(dev), "attention_mask": am[sl].to(dev), "labels": labels[sl].to(dev)}
        tr.train_step([batch])
        if step == 0:
            torch.cuda.synchronize()
            first_grad = (store.grad.float() / world).cpu()
    torch.cuda.synchronize()
    in_sync = params_in_sync(store)
    engine = getattr(buck, "engine", None)
    master = store.master.float().cpu()
    overlap = None
    if buck is not None and os.environ.get("HSD_MGPU_OVERLAP") == "1" and buck.set_timing(True):
        # one more step with the engine's per-bucket HIP events on (after the compared state was taken): the
        # comm / compute overlap report bench.py prints for N > 1
        tr.train_step([batch])
        torch.cuda.synchronize()
        overlap = buck.overlap_report()
        buck.set_timing(False)
    if rank == 0:
        torch.save({"grad0": first_grad, "master": master, "in_sync": in_sync, "world": world,
                    "graphs": len(getattr(tr, "_graphs", {}) or {}), "compression": comp,
                    "rccl_world": int(engine.world) if engine is not None else None,
                    "n_buckets": len(buck.buckets) if buck is not None else 0, "overlap": overlap}, out)
    backend.shutdown()


if __name__ == "__main__":
    main(sys.argv[1])
