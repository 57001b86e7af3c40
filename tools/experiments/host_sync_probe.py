"""Where does the host wait on the GPU inside a training step? bench.py's setup for one config, then (1) the host
enqueue time of each step (no synchronisation: if it is close to the GPU step time the run is host-bound), and (2)
torch's sync debug mode over a few steps, printing the Python stack of every synchronising call.
python tools/host_sync_probe.py --model bert-large-uncased --seq_len 512 --batch_size 8"""
import argparse
import collections
import os
import sys
import time
import traceback
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd import data as hdata  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.train.runner import build  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.utils.args import build_parser  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="bert-large-uncased")
ap.add_argument("--seq_len", type=int, default=512)
ap.add_argument("--batch_size", type=int, default=8)
a = ap.parse_args()
targs, _ = build_parser("train").parse_known_args(
    ["--model_name_or_path", a.model, "--train_batch_size", str(a.batch_size), "--dtype", "bf16",
     "--learning_rate", "5e-5", "--log_every", "0", "--max_seq_length", str(a.seq_len)])
parts = build(targs, "train")
trainer, dev = parts["trainer"], parts["device"]
cfg = parts["model"].cfg
ds = hdata.synthetic_classification(a.batch_size, a.seq_len, cfg.vocab_size, seed=1, full_length=True)
b = {"input_ids": torch.from_numpy(ds.input_ids).long().to(dev),
     "attention_mask": torch.from_numpy(ds.attention_mask).long().to(dev),
     "labels": torch.from_numpy(ds.labels).long().to(dev)}
for _ in range(5):
    trainer.train_step([b])
torch.cuda.synchronize()
host = []
t_all = time.perf_counter()
for _ in range(20):
    t0 = time.perf_counter()
    trainer.train_step([b])
    host.append((time.perf_counter() - t0) * 1e3)
torch.cuda.synchronize()
gpu = (time.perf_counter() - t_all) * 1e3 / 20
host.sort()
print(f"host enqueue ms/step median {host[10]:.2f} min {host[0]:.2f} max {host[-1]:.2f}; wall ms/step {gpu:.2f}",
      flush=True)
seen = collections.Counter()


def show(message, category, filename, lineno, file=None, line=None):
    st = "".join(traceback.format_stack(limit=12)[:-2])
    key = st
    if seen[key] == 0:
        print(f"--- sync: {message}\n{st}", flush=True)
    seen[key] += 1


warnings.showwarning = show
warnings.simplefilter("always")
torch.cuda.set_sync_debug_mode("warn")
for _ in range(3):
    trainer.train_step([b])
torch.cuda.set_sync_debug_mode(0)
torch.cuda.synchronize()
print(f"distinct synchronising call sites: {len(seen)}, calls over 3 steps: {sum(seen.values())}")
