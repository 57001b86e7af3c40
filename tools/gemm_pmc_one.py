"""Run one of the headline layer's GEMMs (tools/gemm_sol.py GEMMS, by name) 10 times: a rocprofv3 --pmc target.
    python tools/gemm_pmc_one.py ffn1_fwd_gelu_d [T]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gemm_sol import GEMMS  # noqa: E402

from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"
name = sys.argv[1]
T = int(sys.argv[2]) if len(sys.argv) > 2 else 131072
rnd = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).bfloat16()  # noqa: E731
(_, lay, M, N, K, epi), = [g for g in GEMMS if g[0] == name]
if lay == "NT":
    M = T
    a, b = rnd(M, K), rnd(N, K) * 0.05
    bias, aux = rnd(N), rnd(M, N)
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    c2 = torch.empty_like(c) if epi in (2, 8) else None
    db = torch.zeros(N, device=dev) if epi in (5, 9) else None
    fn = lambda: C_.gemm2(a, b, c, 0, 0, epi, bias if epi in (1, 2, 3, 8) else None,  # noqa: E731
                          aux if epi in (3, 4, 5, 9) else None, c2, 0.1 if epi == 3 else 0.0, 7, 1, None, db)
else:
    K = T
    dy, x = rnd(K, M), rnd(K, N)
    g = torch.zeros(M, N, device=dev)
    sp = C_.gemm2_splits(M, N, K)
    ws = torch.empty(sp * M * N, device=dev)
    fn = lambda: C_.gemm2(dy, x, g, 1, 1, 7, None, None, None, 0.0, 0, sp, ws, None)  # noqa: E731
for _ in range(10):
    fn()
torch.cuda.synchronize()
