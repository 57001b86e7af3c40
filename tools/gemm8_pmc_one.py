"""The fp8 GEMMs of the roberta-large MLM step (BASELINE config 5, T = B x S = 64 x 512 = 32,768 tokens), one shape per
run, 10 launches each: a rocprofv3 --pmc / --kernel-trace target (tools/pmc_gemm8.sh).

    python tools/gemm8_pmc_one.py NAME [T]

NAME: qkv_fwd <1> (N 3072, K 1024), out_fwd <3> (N 1024, K 1024, dropout + residual), ffn1_fwd <8> (N 4096, K 1024,
GELU' + GELU with the GELU output's fp8 copy for FFN2), ffn2_fwd <3> (N 1024, K 4096), ffn2_dgrad <9> (N 4096, K 1024:
x GELU', bias-gradient sums, fp8 copy for the FFN1 dgrad), qkv_dgrad <4> (N 1024, K 3072, + residual), wgrad_ffn
(the fp8 TT weight gradient of the 1024 x 4096 FFN weight)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C_ = hip._C
dev = "cuda"
SHAPES = {"qkv_fwd": (3072, 1024, 1), "out_fwd": (1024, 1024, 3), "ffn1_fwd": (4096, 1024, 8),
          "ffn2_fwd": (1024, 4096, 3), "ffn2_dgrad": (4096, 1024, 9), "qkv_dgrad": (1024, 3072, 4)}
name = sys.argv[1]
T = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
rnd = lambda *s: (torch.rand(*s, device=dev) * 2 - 1)  # noqa: E731
if name == "wgrad_ffn":
    M, N = 1024, 4096
    qdy, sdy = hip.quant_fp8(rnd(T, M).bfloat16(), 0)
    qx, sx = hip.quant_fp8(rnd(T, N).bfloat16(), 0)
    g = torch.zeros(M, N, device=dev)
    ws = torch.empty(C_.gemm8_wgrad_ws_numel(M, N, T, 0), device=dev)
    fn = lambda: C_.gemm8_wgrad(0, qdy, 0, sdy, qx, 0, sx, g, 0, ws)  # noqa: E731
else:
    N, K, epi = SHAPES[name]
    qa, sa = hip.quant_fp8(rnd(T, K).bfloat16(), 0)
    qb, sb = hip.quant_fp8((rnd(N, K) * 0.05).bfloat16(), 0)
    bias, aux = rnd(N).bfloat16(), rnd(T, N).bfloat16()
    y = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
    y2 = torch.empty_like(y) if epi in (2, 8) else None
    db = torch.zeros(N, device=dev) if epi == 9 else None
    kw = {}
    if epi in (8, 9):  # the step's fused fp8 copy of the output for the next fp8 GEMM (delayed-scaling site)
        st = torch.tensor([3.0, 0.0], device=dev)
        kw = dict(q8=torch.empty(T, N, dtype=torch.uint8, device=dev), q8_amax=st[0:1],
                  q8_sinv=torch.empty(1, device=dev), q8_track=st[1:2], q8fmt=0)
    fn = lambda: C_.gemm8(qa, 0, sa, qb, 0, sb, y, epi, bias if epi in (1, 2, 3, 8) else None,  # noqa: E731
                          aux if epi in (3, 4, 5, 9) else None, y2, 0.1 if epi == 3 else 0.0, 7, db, **kw)
for _ in range(10):
    fn()
torch.cuda.synchronize()
print(name, "ok")
