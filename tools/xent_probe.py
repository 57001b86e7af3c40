"""Cross-entropy kernel (xent.hip) on the MLM head's logits shape: time per call and bytes/s.
python tools/xent_probe.py [rows] [V]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

dev = "cuda"
R = int(sys.argv[1]) if len(sys.argv) > 1 else 4928
V = int(sys.argv[2]) if len(sys.argv) > 2 else 50265
Vp = -(-V // 256) * 256
logits = torch.randn(R, Vp, device=dev).bfloat16()
labels = torch.randint(0, V, (R,), device=dev)
dl = torch.empty_like(logits)
stats = torch.zeros(2, device=dev)
nv = torch.full((1,), float(R), device=dev)
f = lambda: hip._C.xent(logits, labels, dl, stats, nv, V)  # noqa: E731
for _ in range(3):
    f()
torch.cuda.synchronize()
ts = []
for _ in range(10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    f()
    e.record()
    e.synchronize()
    ts.append(s.elapsed_time(e) * 1e3)
ts.sort()
t = ts[5]
print(json.dumps({"rows": R, "V": V, "us": round(t, 1), "TBps_3pass": round(3 * R * Vp * 2 / t / 1e6, 2)}))
