"""Per-step fp8 weight-copy refresh (FlatParamStore.refresh_fp8: amax_many + quant_many over the encoder weights) of
roberta-large in isolation: us per refresh and effective TB/s.   python tools/fp8_refresh_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.models.bert import build_model  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.models.config import resolve_config  # noqa: E402
from huggingface_sagemaker_tensorflow_distributed_amd.parallel import FlatParamStore  # noqa: E402

dev = torch.device("cuda", 0)
m = build_model(resolve_config("roberta-large"), task="masked-lm", seed=0).to(dev)
store = FlatParamStore(m, dev, compute_dtype=torch.bfloat16, fp8=True)
n = sum(int(d[2]) for d in store._fp8_desc[0].cpu().tolist())  # weights (the quant pass writes W8 and W8ᵀ)
for _ in range(3):
    store.refresh_fp8()
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = []
for _ in range(3):
    a.record()
    for _ in range(10):
        store.refresh_fp8()
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b) / 10 * 1e3)
us = min(ts)
print(f"HSD_FP8_SLOT={os.environ.get('HSD_FP8_SLOT', '32')} refresh_fp8: {us:.1f} us for {n / 1e6:.1f} M weights "
      f"(amax reads W 2 B, quant reads W and Wt 4 B and writes 2 B per weight: {8 * n / us / 1e6:.2f} TB/s)", flush=True)
