"""Debug the whole-step HIP graph: finiteness of weights / grads / loss around capture and each replay."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model, resolve_config  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.optim import FusedAdam  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.train.trainer import Trainer  # noqa: E402

gpu = torch.device("cuda", 0)
cfg = resolve_config("bert-base-uncased").replace(num_hidden_layers=2)
model = build_model(cfg, seed=0).to(gpu)
model.rng.base_seed = 5
store = FlatParamStore(model, gpu, compute_dtype=torch.bfloat16)
opt = FusedAdam(store, lr=1e-4)
tr = Trainer(model, store, opt, None, gpu, hip_graph=True)
print("full", tr._full_graph, "overlap", tr._opt_overlap)
g = torch.Generator().manual_seed(0)
ids = torch.randint(1000, 30000, (16, 128), generator=g)
mb = {"input_ids": ids.to(gpu), "attention_mask": torch.ones(16, 128, dtype=torch.long, device=gpu),
      "labels": torch.randint(0, 2, (16,), generator=g).to(gpu)}


def fin(tag):
    torch.cuda.synchronize()
    print(tag, "master", bool(torch.isfinite(store.master).all()), "compute", bool(torch.isfinite(store.compute).all()),
          "grad", bool(torch.isfinite(store.grad).all()), float(store.grad.abs().max()),
          "m", bool(torch.isfinite(opt.exp_avg).all()), "dcoef", opt.dcoef.tolist() if opt.dcoef is not None else None,
          flush=True)


import threading  # noqa: E402

ov = tr._opt_overlap
_orig = ov.mark_ready
seen = []


def traced(i):
    if len(seen) < 6:
        seen.append((i, threading.current_thread().name, torch.cuda.current_stream().cuda_stream,
                     torch.cuda.is_current_stream_capturing(), opt._began))
    _orig(i)


store.ready_callback = traced
fin("init")
cs = tr._full_graph_for(mb)
fin("after capture")
print("hook calls during capture:", seen, "ov stream", ov.stream.cuda_stream)
print("static loss before replay", float(cs.loss))
for i in range(3):
    tr._seed.set_step(i)
    loss, _ = cs.run(mb)
    torch.cuda.synchronize()
    print("replay", i, "loss", float(loss), flush=True)
    fin(f"after replay {i}")
