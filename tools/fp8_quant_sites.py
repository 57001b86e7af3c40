"""Which fp8 sites still run the standalone quantiser in a calibrated step? Runs a few fp8 training steps of the given
model / task and prints, for the last step, every fp8_quant call with the Python frames that issued it.

    python tools/fp8_quant_sites.py [--model roberta-large] [--task masked-lm] [--layers 2] [--seq_len 512] [--batch 8]"""
import argparse
import collections
import os
import sys
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd import data as hdata  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.models import build_model, resolve_config  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="roberta-large")
ap.add_argument("--task", default="masked-lm")
ap.add_argument("--layers", type=int, default=2)
ap.add_argument("--seq_len", type=int, default=512)
ap.add_argument("--batch", type=int, default=8)
a = ap.parse_args()
dev = torch.device("cuda", 0)
cfg = resolve_config(a.model).replace(num_hidden_layers=a.layers)
if a.task == "masked-lm":
    ds = hdata.synthetic_mlm(a.batch, a.seq_len, cfg.vocab_size, seed=3)
else:
    ds = hdata.synthetic_classification(a.batch, a.seq_len, cfg.vocab_size, seed=3, full_length=True)
ids = torch.from_numpy(ds.input_ids).long().to(dev)
am = torch.from_numpy(ds.attention_mask).long().to(dev)
labels = torch.from_numpy(ds.labels).long().to(dev)
m = build_model(cfg, task=a.task, seed=0).to(dev)
store = FlatParamStore(m, dev, compute_dtype=torch.bfloat16, fp8=True)
hip.set_fp8(True)
orig = hip._C
sites = collections.Counter()


class _Spy:
    def __getattr__(self, k):
        f = getattr(orig, k)
        if k not in ("fp8_quant", "fp8_quant_many"):
            return f

        def w(*args, **kw):
            st = traceback.extract_stack()[:-1]
            key = " <- ".join(f"{os.path.basename(fr.filename)}:{fr.lineno}:{fr.name}" for fr in st[-5:][::-1])
            sites[(k, key)] += 1
            return f(*args, **kw)
        return w


for step in range(4):
    if step == 3:
        hip._C = _Spy()
    m.train()
    m.rng.new_step(step)
    store.zero_grad()
    loss, _ = m(ids, attention_mask=am, labels=labels)
    loss.backward()
    torch.cuda.synchronize()
    hip._C = orig
    store.refresh_fp8()
print(f"calibrated step ({a.layers} layers): {sum(sites.values())} standalone quantiser calls")
for (k, key), n in sites.most_common():
    print(f"{n:4d}  {k}  {key}")
