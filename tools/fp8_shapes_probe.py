"""fp8 (gemm8pk) vs bf16 (gemm2) NT GEMMs on the roberta-large MLM S=512 B=64 shapes (T = 32768), in isolation.
    python tools/fp8_shapes_probe.py [T]  -> one JSON line per GEMM (us, TFLOP/s)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from huggingface_sagemaker_tensorflow_distributed_amd.ops import hip  # noqa: E402

C = hip._C
dev = "cuda"
T = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
H, F = 1024, 4096
SHAPES = [("qkv_fwd", 3 * H, H, 1), ("out_fwd", H, H, 3), ("ffn1_fwd", F, H, 8), ("ffn2_fwd", H, F, 3),
          ("ffn2_dgrad", F, H, 9), ("ffn1_dgrad", H, F, 4), ("out_dgrad", H, H, 0), ("qkv_dgrad", H, 3 * H, 4)]


def timeit(fn, iters=10):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e3


for name, N, K, epi in SHAPES:
    x = (torch.randn(T, K, device=dev)).bfloat16()
    w = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
    bias = torch.randn(N, device=dev).bfloat16()
    aux = torch.randn(T, N, device=dev).bfloat16()
    y = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
    y2 = torch.empty_like(y) if epi == 8 else None
    db = torch.zeros(N, device=dev) if epi == 9 else None
    qx, sx = hip.quant_fp8(x, 0)
    qw, sw = hip.quant_fp8(w, 0)
    b_ = bias if epi in (1, 3, 8) else None
    a_ = aux if epi in (3, 4, 9) else None
    t16 = min(timeit(lambda: C.gemm2(x, w, y, 0, 0, epi, b_, a_, y2, 0.1 if epi == 3 else 0.0, 7, 0, None, db))
              for _ in range(3))
    t8 = min(timeit(lambda: C.gemm8(qx, 0, sx, qw, 0, sw, y, epi, b_, a_, y2, 0.1 if epi == 3 else 0.0, 7, db))
             for _ in range(3))
    fl = 2.0 * T * N * K
    print(json.dumps({"gemm": name, "M": T, "N": N, "K": K, "epi": epi, "bf16_us": round(t16, 1), "fp8_us": round(t8, 1),
                      "bf16_TF": round(fl / t16 / 1e6, 1), "fp8_TF": round(fl / t8 / 1e6, 1),
                      "speedup": round(t16 / t8, 3)}), flush=True)
