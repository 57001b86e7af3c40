"""Run one gemm2 configuration repeatedly (rocprofv3 PMC target).  python tools/gemm2_one.py {fwd|gelu|dgelu|wgrad|wgrad_out}"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
T = int(os.environ.get("G1_T", "32768"))
which = sys.argv[1] if len(sys.argv) > 1 else "fwd"
N, K = (3072, 768) if which in ("fwd", "gelu", "dgelu", "wgrad") else (768, 768)
x = torch.randn(T, K, device="cuda").bfloat16()
w = torch.randn(N, K, device="cuda").bfloat16()
b = torch.randn(N, device="cuda").bfloat16()
y = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
y2 = torch.empty_like(y)
dy = torch.randn(T, N, device="cuda").bfloat16()
gw = torch.zeros(N, K, device="cuda")
sp = C_.gemm2_splits(N, K, T)
ws = torch.empty(sp * N * K, device="cuda")
w2t = torch.randn(N, K, device="cuda").bfloat16()  # dgelu: dx[T][N] = dy2[T][K] . w2t^T
dy2 = torch.randn(T, K, device="cuda").bfloat16()
for _ in range(10):
    if which == "fwd":
        C_.gemm2(x, w, y, 0, 0, 0, None, None, None, 0.0, 0, 1, None, None)
    elif which == "gelu":
        C_.gemm2(x, w, y, 0, 0, 2, b, None, y2, 0.0, 0, 1, None, None)
    elif which == "dgelu":
        C_.gemm2(dy2, w2t, y, 0, 0, 5, None, y2, None, 0.0, 0, 1, None, None)
    else:
        C_.gemm2(dy, x, gw, 1, 1, 7, None, None, None, 0.0, 0, sp, ws, None)
torch.cuda.synchronize()
