"""Host-side (Python) cost of a training step at a small batch: cProfile over N steps after warm-up.
    python tools/cpu_profile_step.py [--model M] [--seq_len S] [--batch_size B]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd import data as hdata  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.train.runner import build  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.utils.args import build_parser  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="bert-base-uncased")
ap.add_argument("--seq_len", type=int, default=128)
ap.add_argument("--batch_size", type=int, default=32)
ap.add_argument("--steps", type=int, default=20)
a = ap.parse_args()
args, _ = build_parser("train").parse_known_args(
    ["--model_name_or_path", a.model, "--train_batch_size", str(a.batch_size), "--dtype", "bf16",
     "--max_seq_length", str(a.seq_len), "--log_every", "0"])
parts = build(args, "train")
tr = parts["trainer"]
dev = tr.device
ds = hdata.synthetic_classification(a.batch_size, a.seq_len, parts["model"].cfg.vocab_size, seed=0)
mb = {"input_ids": torch.from_numpy(ds.input_ids).long().to(dev),
      "attention_mask": torch.from_numpy(ds.attention_mask).long().to(dev),
      "labels": torch.from_numpy(ds.labels).long().to(dev)}
for _ in range(5):
    tr.train_step([mb])
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.steps):
    tr.train_step([mb])
t_host = time.perf_counter() - t0
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
print(f"host issue time {1e3 * t_host / a.steps:.2f} ms/step, wall {1e3 * t_all / a.steps:.2f} ms/step")
pr = cProfile.Profile()
pr.enable()
for _ in range(a.steps):
    tr.train_step([mb])
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(20)

# the backward runs on autograd's device thread: profile it there by wrapping every custom Function's backward
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip as _hip  # noqa: E402

bpr = cProfile.Profile()
for name in dir(_hip):
    obj = getattr(_hip, name)
    if isinstance(obj, type) and issubclass(obj, torch.autograd.Function) and "backward" in obj.__dict__:
        orig = obj.__dict__["backward"].__func__

        def wrap(orig):
            def bw(ctx, *g):
                bpr.enable()
                try:
                    return orig(ctx, *g)
                finally:
                    bpr.disable()
            return staticmethod(bw)

        setattr(obj, "backward", wrap(orig))
for _ in range(a.steps):
    tr.train_step([mb])
torch.cuda.synchronize()
print("==== backward (autograd thread)")
pstats.Stats(bpr).sort_stats("tottime").print_stats(30)
