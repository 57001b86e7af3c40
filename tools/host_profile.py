"""Host-side cost of one training step (is the eager step launch-bound?): builds the bench's trainer, then per step
(a) host issue time of train_step from an idle GPU (synchronize before), (b) the time until the GPU drains, and a
cProfile of the issue path (top functions by own time).

    python tools/host_profile.py [bench.py-style args: --model ... --seq_len ... --batch_size ... --dtype ...]"""
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd import data as hdata  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.train.runner import build  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.utils.args import build_parser  # noqa: E402

args = dict(model="bert-large-uncased", seq_len="512", batch_size="8", dtype="bf16", hip_graph="false")
av = sys.argv[1:]
for i in range(0, len(av), 2):
    args[av[i].lstrip("-")] = av[i + 1]
targs, _ = build_parser("train").parse_known_args(
    ["--model_name_or_path", args["model"], "--train_batch_size", args["batch_size"], "--dtype", args["dtype"],
     "--hip_graph", args["hip_graph"], "--learning_rate", "5e-5", "--log_every", "0", "--max_seq_length",
     args["seq_len"]])
parts = build(targs, "train")
trainer, dev = parts["trainer"], parts["device"]
cfg = parts["model"].cfg
B, S = int(args["batch_size"]), int(args["seq_len"])
ds = hdata.synthetic_classification(B, S, cfg.vocab_size, seed=1, full_length=True)
mb = {"input_ids": torch.from_numpy(ds.input_ids).long().to(dev),
      "attention_mask": torch.from_numpy(ds.attention_mask).long().to(dev),
      "labels": torch.from_numpy(ds.labels).long().to(dev)}
for _ in range(5):
    trainer.train_step([mb])
torch.cuda.synchronize()
issue, total = [], []
for _ in range(10):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    trainer.train_step([mb])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    issue.append((t1 - t0) * 1e3)
    total.append((t2 - t0) * 1e3)
issue.sort()
total.sort()
print(f"host issue ms/step (from idle GPU): median {issue[5]:.2f} min {issue[0]:.2f}; issue + drain: median "
      f"{total[5]:.2f} min {total[0]:.2f}", flush=True)
# back-to-back steps (the bench's loop)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    trainer.train_step([mb])
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"back-to-back: host returns after {(t1 - t0) * 50:.2f} ms/step, GPU done {(t2 - t0) * 50:.2f} ms/step", flush=True)
pr = cProfile.Profile()
torch.cuda.synchronize()
pr.enable()
for _ in range(5):
    trainer.train_step([mb])
pr.disable()
torch.cuda.synchronize()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(35)
print(s.getvalue()[:9000])
