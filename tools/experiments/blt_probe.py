"""hipBLASLt's kernel choice for the BERT-base B=1024 GEMM shapes (run under rocprofv3 --kernel-trace --stats)."""
import sys

import torch

T = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
for name, (N, K) in {"qkv": (2304, 768), "out": (768, 768), "ffn1": (3072, 768), "ffn2": (768, 3072)}.items():
    x = torch.randn(T, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    for _ in range(3):
        torch.mm(x, w.t())
torch.cuda.synchronize()
