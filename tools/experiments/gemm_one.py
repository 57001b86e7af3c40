"""Run a single GEMM config repeatedly (for rocprofv3 counter collection)."""
import sys

import torch

sys.path.insert(0, ".")
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
T, N, K = 32768, 3072, 768
which = sys.argv[1] if len(sys.argv) > 1 else "fwd"
x = torch.randn(T, K, device="cuda").bfloat16()
w = torch.randn(N, K, device="cuda").bfloat16()
dy = torch.randn(T, N, device="cuda").bfloat16()
y = torch.empty(T, N, device="cuda", dtype=torch.bfloat16)
dx = torch.empty(T, K, device="cuda", dtype=torch.bfloat16)
gw = torch.zeros(N, K, device="cuda")
for _ in range(10):
    if which == "fwd":
        C_.gemm_variant(x, w, y, 0, 0, 0)
    elif which == "fwd128":
        C_.gemm_variant(x, w, y, 0, 0, 5)
    elif which == "dgrad":
        C_.gemm_variant(dy, w, dx, 0, 1, 3)
    elif which == "wgrad":
        C_.gemm(dy, x, gw, 1, 1, 6, None, None, None, 0.0, 0, 8)
    elif which == "torch":
        torch.addmm(w[:, 0], x, w.t())
torch.cuda.synchronize()
